// Loader / decoder split probe (diagnostic, not product; round 6): config 2's traffic (per
// 64-packet tile 4 KiB of packet bytes, 64 offsets + 64 caplens from their own arrays, two 16-B
// result stores per lane) with ONE loader wave per workgroup streaming tiles into an LDS ring by
// LDS-DMA (P tiles in flight, a steady request stream) and the other waves decoding from the ring
// (an emulated decode of SPIN dependent steps).  Flags in LDS: ready[slot] = tile + 1 once its
// bytes landed, freed[slot] = the slot's use count once its decoder is done.  Every spin loop is
// capped (err[0] counts the caps hit), so the kernel always drains.
//   hipcc --offload-arch=gfx950 -O3 -o stream_split stream_split.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

extern __shared__ __attribute__((aligned(16))) uint8_t g_lds[];

__device__ __forceinline__ void glds16(const void *gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}
__device__ __forceinline__ void glds4(const void *gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %2 nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vmwait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int SPIN>
__device__ __forceinline__ uint32_t fake_decode(uint32_t pkt, uint32_t o, uint32_t c) {
  uint32_t a = *reinterpret_cast<const uint32_t *>(g_lds + pkt + 12);
  uint32_t b = *reinterpret_cast<const uint32_t *>(g_lds + pkt + 24);
  uint32_t d = *reinterpret_cast<const uint32_t *>(g_lds + pkt + 36);
  uint32_t x = a ^ (b << 1) ^ (d >> 3) ^ o ^ c;
#pragma unroll 1
  for (int s = 0; s < SPIN; s++) x = __builtin_amdgcn_alignbyte(x, x * 0x9E3779B1u + (uint32_t)s, 3);
  return x;
}

constexpr uint32_t kSlot = 4096u + 512u;
constexpr uint32_t kSpinCap = 1u << 22;

__device__ __forceinline__ uint32_t *lds_word(uint32_t a) {
  return static_cast<uint32_t *>(__builtin_assume_aligned(g_lds + a, 4));
}
__device__ __forceinline__ uint32_t lds_ld(uint32_t a) {
  return __hip_atomic_load(lds_word(a), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t a, uint32_t v) {
  __hip_atomic_store(lds_word(a), v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int NW, int R, int P, int SPIN, int SH = 0>
__global__ __launch_bounds__(64 * NW) void split_k(const uint8_t *__restrict__ data, const uint32_t *__restrict__ off,
                                                   const uint32_t *__restrict__ cap, v4u *rec, uint32_t ntiles,
                                                   uint32_t *err) {
  static_assert(R > P, "ring");
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ready = R * kSlot, freed = ready + 4u * R;
  if (threadIdx.x < 2u * R) reinterpret_cast<uint32_t *>(g_lds + ready)[threadIdx.x] = 0u;
  __syncthreads();
  const uint32_t G = ntiles > blockIdx.x ? (ntiles - blockIdx.x + gridDim.x - 1u) / gridDim.x : 0u;
  if (wave == 0) {  // the loader
    uint32_t issued = 0, signaled = 0;
    auto signal_all = [&] {
      vmwait<0>();
      for (; signaled < issued; signaled++)
        if (lane == 0u) lds_st(ready + 4u * (signaled % R), signaled + 1u);
    };
    for (uint32_t g = 0; g < G; g++) {
      const uint32_t slot = g % R;
      if (g >= R) {
        uint32_t spins = 0;
        if (lds_ld(freed + 4u * slot) < g / R) {
          signal_all();  // whatever landed, so that the decoders can free slots
          while (lds_ld(freed + 4u * slot) < g / R && ++spins < kSpinCap) __builtin_amdgcn_s_sleep(1);
          if (spins >= kSpinCap && lane == 0u) atomicAdd(err, 1u);
        }
      }
      const uint32_t t = blockIdx.x + g * gridDim.x, b = slot * kSlot;
#pragma unroll
      for (int j = 0; j < 4; j++)  // SH: the window's source shifted back by SH bytes (misaligned DMA);
        // the scalar base moves, never the lane offset, and the batch's first chunk is not shifted
        glds16(data + (uint64_t)t * 4096u + 1024u * j - ((t != 0u || j != 0) ? (uint32_t)SH : 0u), 16u * lane,
               b + 1024u * j);
      glds4(off + t * 64u, 4u * lane, b + 4096u);
      glds4(cap + t * 64u, 4u * lane, b + 4096u + 256u);
      issued++;
      if (issued - signaled >= (uint32_t)P) {  // the oldest in flight has landed
        vmwait<6 * (P - 1)>();
        if (lane == 0u) lds_st(ready + 4u * (signaled % R), signaled + 1u);
        signaled++;
      }
    }
    signal_all();
    return;
  }
  const uint32_t D = NW - 1, d = wave - 1;
  for (uint32_t g = d; g < G; g += D) {
    const uint32_t slot = g % R, b = slot * kSlot;
    uint32_t spins = 0;
    while (lds_ld(ready + 4u * slot) != g + 1u && ++spins < kSpinCap) __builtin_amdgcn_s_sleep(1);
    if (spins >= kSpinCap && lane == 0u) atomicAdd(err, 1u);
    const uint32_t o = *reinterpret_cast<const uint32_t *>(g_lds + b + 4096u + 4u * lane);
    const uint32_t c = *reinterpret_cast<const uint32_t *>(g_lds + b + 4096u + 256u + 4u * lane);
    const uint32_t x = fake_decode<SPIN>(b + 64u * lane + (o & 15u), o, c);
    if (SH) {  // LDS byte 16 l + 5 holds global byte 4096 t + 16 l + 5 - SH (data[i] = i mod 251)
      const uint32_t t = blockIdx.x + g * gridDim.x;
      const uint32_t want = (uint32_t)(((uint64_t)t * 4096u + 16u * lane + 5u - SH) % 251u);
      if (t != 0u && g_lds[b + 16u * lane + 5u] != want) atomicAdd(err + 1, 1u);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0u) lds_st(freed + 4u * slot, g / R + 1u);
    const uint64_t i = (uint64_t)(blockIdx.x + g * gridDim.x) * 64u + lane;
    __builtin_nontemporal_store(v4u{x, x ^ 1u, x * 3u, 0u}, rec + 2 * i);
    __builtin_nontemporal_store(v4u{x * 5u, 0u, x * 7u, 0u}, rec + 2 * i + 1);
  }
}

template <typename L>
static float timeit(L launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 300; r++) launch();
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++) launch();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  CK(hipGetLastError());
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

template <int NW, int R, int P, int SPIN, int SH = 0>
static void one(const char *nm, int cus, int wpc, const uint8_t *data, const uint32_t *off, const uint32_t *cap,
                v4u *rec, uint32_t ntiles, uint32_t *err, int reps) {
  const size_t lds = (size_t)R * kSlot + 8u * R;
  const double bytes = (double)ntiles * 64.0 * (72.0 + 32.0);
  CK(hipMemset(err, 0, 8));
  const float ms = timeit([&] {
    hipLaunchKernelGGL((split_k<NW, R, P, SPIN, SH>), dim3(cus * wpc), dim3(64 * NW), lds, 0, data, off, cap, rec, ntiles, err);
  }, reps);
  uint32_t e[2] = {0, 0};
  CK(hipMemcpy(e, err, 8, hipMemcpyDeviceToHost));
  printf("RESULT spin=%d %-14s sh=%d wpc=%d ms=%.4f TBps=%.3f caps=%u mismatches=%u\n", SPIN, nm, SH, wpc, ms,
         bytes / (ms * 1e-3) / 1e12, e[0], e[1]);
  fflush(stdout);
}

template <int SPIN>
static void run(int cus, const uint8_t *data, const uint32_t *off, const uint32_t *cap, v4u *rec, uint32_t ntiles,
                uint32_t *err, int reps) {
  one<8, 12, 3, SPIN>("nw8_r12_p3", cus, 2, data, off, cap, rec, ntiles, err, reps);
  one<8, 12, 3, SPIN, 2>("nw8_r12_p3", cus, 2, data, off, cap, rec, ntiles, err, reps);
  one<8, 12, 4, SPIN>("nw8_r12_p4", cus, 2, data, off, cap, rec, ntiles, err, reps);
  one<16, 24, 8, SPIN>("nw16_r24_p8", cus, 1, data, off, cap, rec, ntiles, err, reps);
  one<16, 24, 8, SPIN, 2>("nw16_r24_p8", cus, 1, data, off, cap, rec, ntiles, err, reps);
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("stream_split: %s %d CUs\n", prop.gcnArchName, cus);
  const uint32_t ntiles = 1u << 18;
  const uint64_t n = (uint64_t)ntiles * 64u;
  uint8_t *data = nullptr;
  uint32_t *off = nullptr, *cap = nullptr, *err = nullptr;
  v4u *rec = nullptr;
  CK(hipMalloc(&data, n * 64u));
  {
    uint8_t *h = (uint8_t *)malloc(n * 64u);
    for (uint64_t i = 0; i < n * 64u; i++) h[i] = (uint8_t)(i % 251u);
    CK(hipMemcpy(data, h, n * 64u, hipMemcpyHostToDevice));
    free(h);
  }
  CK(hipMalloc(&off, n * 4u));
  CK(hipMalloc(&cap, n * 4u));
  CK(hipMemset(off, 0, n * 4u));
  CK(hipMemset(cap, 0x40, n * 4u));
  CK(hipMalloc(&rec, n * 32u));
  CK(hipMalloc(&err, 8));
  run<0>(cus, data, off, cap, rec, ntiles, err, reps);
  run<64>(cus, data, off, cap, rec, ntiles, err, reps);
  run<128>(cus, data, off, cap, rec, ntiles, err, reps);
  run<160>(cus, data, off, cap, rec, ntiles, err, reps);
  CK(hipFree(data));
  CK(hipFree(off));
  CK(hipFree(cap));
  CK(hipFree(rec));
  CK(hipFree(err));
  return 0;
}
