// F3 floor probe (diagnostic, not product; VERDICT r04 "Next round" item 5): what do the
// memory-side atomics of an existing-flow insert cost by themselves?  gpd_flow.hip's insert
// of a packet whose flow already has a record issues two device-scope atomics on the record's
// 64-B hot line: the packed packets|bytes atomicAdd (its old word returned, for the carry
// rule) and atomicMax of `last`.  Here: a table of 2^25 slots of 64 B (the
// bench's table for 2^24 flows at load 1/2), 2^24 packets, each on its own random line
// (slot = i * odd mod 2^25: a bijection, every line touched once per launch, as the bench's
// "every packet an existing flow" case does), no decode, no probe, no key compare.
//   two_atomics   : atomicAdd (returning) + atomicMax on the same line   <- the verdict's probe
//   two_noret     : both atomics without using the returned value
//   one_atomic    : the returning atomicAdd only
//   read_line     : one 64-B read of the line (a 16-B load per lane for 4 lanes) and nothing else
//   read_two      : that read, then the two atomics (the insert's minimum for an existing flow)
//   hipcc --offload-arch=gfx950 -O3 -o atomic_floor atomic_floor.hip && ./atomic_floor
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr uint32_t kSlotsLog = 25;
constexpr uint64_t kSlots = 1ull << kSlotsLog;
constexpr uint64_t kPkts = 1ull << 24;
constexpr uint32_t kWords = 8;  // a slot: 8 x u64 = 64 B

__device__ __forceinline__ uint64_t slot_of(uint64_t i) {
  return (i * 0x9E3779B97F4A7C15ull) & (kSlots - 1);  // odd multiplier: a bijection mod 2^25
}

enum Mode { kTwo = 0, kTwoNoRet = 1, kOne = 2, kRead = 3, kReadTwo = 4 };

template <int MODE>
__global__ __launch_bounds__(256) void probe_k(unsigned long long *tab, uint64_t n, uint64_t seq,
                                               unsigned long long *sink) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    unsigned long long *line = tab + slot_of(i) * kWords;
    if (MODE == kRead || MODE == kReadTwo) {
      // the hot record's fingerprint + key words (what the insert compares), as 4 x 16 B
      const ulonglong2 *q = reinterpret_cast<const ulonglong2 *>(line);
      const ulonglong2 a = q[0], b = q[1], c = q[2], d = q[3];
      acc ^= a.x ^ a.y ^ b.x ^ b.y ^ c.x ^ c.y ^ d.x ^ d.y;
    }
    if (MODE == kTwo || MODE == kReadTwo) {
      acc += atomicAdd(line + 6, (1ull << 40) | 64ull);
      atomicMax(line + 7, (unsigned long long)(seq + i));
    } else if (MODE == kTwoNoRet) {
      atomicAdd(line + 6, (1ull << 40) | 64ull);
      atomicMax(line + 7, (unsigned long long)(seq + i));
    } else if (MODE == kOne) {
      acc += atomicAdd(line + 6, (1ull << 40) | 64ull);
    }
  }
  if (acc == 0x0123456789ABCDEFull) sink[0] = acc;  // keeps the returned values live
}

template <int MODE>
static float run(unsigned long long *tab, unsigned long long *sink, int blocks, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL(probe_k<MODE>, dim3(blocks), dim3(256), 0, 0, tab, kPkts, 0ull, sink);  // warm
  CK(hipDeviceSynchronize());
  float best = 1e30f, sum = 0;
  for (int r = 0; r < reps; r++) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe_k<MODE>, dim3(blocks), dim3(256), 0, 0, tab, kPkts, (uint64_t)(r + 1) << 24, sink);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
    sum += ms;
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  printf("  mean %.4f ms  best %.4f ms  (%d reps)\n", sum / reps, best, reps);
  return sum / reps;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  unsigned long long *tab = nullptr, *sink = nullptr;
  CK(hipMalloc(&tab, kSlots * 64));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(tab, 0, kSlots * 64));
  printf("atomic_floor: %s, %d CUs; table 2^%u slots x 64 B (%.1f GiB), %llu packets\n", prop.gcnArchName,
         prop.multiProcessorCount, kSlotsLog, kSlots * 64.0 / (1 << 30), (unsigned long long)kPkts);
  for (int bpc : {8, 32}) {
    const int blocks = prop.multiProcessorCount * bpc;
    printf("grid %d workgroups of 256\n", blocks);
    const char *names[] = {"two_atomics", "two_noret", "one_atomic", "read_line", "read_two"};
    float t[5];
    printf("%s\n", names[0]); t[0] = run<kTwo>(tab, sink, blocks, reps);
    printf("%s\n", names[1]); t[1] = run<kTwoNoRet>(tab, sink, blocks, reps);
    printf("%s\n", names[2]); t[2] = run<kOne>(tab, sink, blocks, reps);
    printf("%s\n", names[3]); t[3] = run<kRead>(tab, sink, blocks, reps);
    printf("%s\n", names[4]); t[4] = run<kReadTwo>(tab, sink, blocks, reps);
    for (int k = 0; k < 5; k++) {
      const double reqs = (k == 2 || k == 3) ? 1.0 : 2.0;
      printf("RESULT grid=%d %s ms=%.4f Gpkt/s=%.2f G_atomic/s=%.2f\n", blocks, names[k], t[k],
             kPkts / (t[k] * 1e6), k == 3 ? 0.0 : kPkts * (k == 4 ? 2.0 : reqs) / (t[k] * 1e6));
    }
  }
  CK(hipFree(tab));
  CK(hipFree(sink));
  return 0;
}
