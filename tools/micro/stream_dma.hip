// Streaming-structure probe for config 2 (diagnostic, not product; round 6):
// the decode kernel's real traffic (per 64-packet tile: 4 KiB of packet bytes, 64 u32 offsets
// and 64 u32 caplens from their own arrays, two 16-B result stores per lane) moved by
//   reg  : rs_kernel's structure — the next tile's window in VGPRs (one window in flight per
//          wave), committed to LDS with ds_write_b128, descriptors two tiles ahead in VGPRs;
//   dmaN : LDS-DMA (global_load_lds_dwordx4 / _dword) into N buffers per wave, N-1 tiles in
//          flight, every wait an explicit counted vmcnt;
// with an emulated decode: SPIN dependent VALU steps on three LDS words of the lane's packet.
// At 2, 3 and 4 workgroups (of 4 waves) per CU.  Does keeping two or three windows in flight
// per wave at 2 workgroups per CU reach the 2-workgroup streaming rate (tile_map.log 0.2975 ms)?
//   hipcc --offload-arch=gfx950 -O3 -o stream_dma stream_dma.hip
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
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// the emulated decode: three LDS words of the lane's packet, SPIN dependent steps
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

__device__ __forceinline__ void store_rec(v4u *rec, uint64_t i, uint32_t x) {
  __builtin_nontemporal_store(v4u{x, x ^ 1u, x * 3u, 0u}, rec + 2 * i);
  __builtin_nontemporal_store(v4u{x * 5u, 0u, x * 7u, 0u}, rec + 2 * i + 1);
}

// rs_kernel's structure (4 KiB windows in VGPRs, single LDS buffer)
template <int SPIN, bool WAITST = false>
__global__ __launch_bounds__(256) void reg_k(const uint8_t *__restrict__ data, const uint32_t *__restrict__ off,
                                             const uint32_t *__restrict__ cap, v4u *rec, uint32_t ntiles) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  const uint32_t buf = wave * 4096u;
  uint32_t t = blockIdx.x * 4u + wave;
  if (t >= ntiles) return;
  auto dl = [&](uint32_t u, uint32_t &o, uint32_t &c) {
    o = c = 0;
    if (u < ntiles) {
      o = __builtin_nontemporal_load(off + u * 64u + lane);
      c = __builtin_nontemporal_load(cap + u * 64u + lane);
    }
  };
  v4u wv[4];
  auto wl = [&](uint32_t u) {
#pragma unroll
    for (int j = 0; j < 4; j++)
      wv[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(data + (uint64_t)u * 4096u + 1024u * j + 16u * lane));
    __builtin_amdgcn_sched_barrier(0);
  };
  uint32_t o0, c0, o1, c1, o2, c2;
  dl(t, o0, c0);
  dl(t + nw, o1, c1);
  dl(t + 2 * nw, o2, c2);
  wl(t);
  for (;;) {
    if (WAITST) vmwait<0>();  // (the production kernel's conservative wait: stores included)
#pragma unroll
    for (int j = 0; j < 4; j++) *reinterpret_cast<v4u *>(g_lds + buf + 1024u * j + 16u * lane) = wv[j];
    const uint32_t tn = t + nw;
    if (tn < ntiles) wl(tn);
    const uint32_t x = fake_decode<SPIN>(buf + 64u * lane + (o0 & 15u), o0, c0);
    store_rec(rec, (uint64_t)t * 64u + lane, x);
    if (tn >= ntiles) break;
    t = tn;
    o0 = o1; c0 = c1; o1 = o2; c1 = c2;
    dl(t + 2 * nw, o2, c2);
  }
}


// Two of the wave's tiles per iteration (tiles t and t + nw: two 4 KiB windows, 8 register chunks
// per lane), one pair in flight: twice the bytes per wave-iteration of reg_k.
template <int SPIN>
__global__ __launch_bounds__(256) void reg2_k(const uint8_t *__restrict__ data, const uint32_t *__restrict__ off,
                                              const uint32_t *__restrict__ cap, v4u *rec, uint32_t ntiles) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  const uint32_t buf = wave * 8192u;
  uint32_t t = blockIdx.x * 4u + wave;
  if (t >= ntiles) return;
  v4u wv[8];
  auto wl = [&](uint32_t u) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const uint32_t uu = u + (j >> 2) * nw;
      wv[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(data + (uint64_t)(uu < ntiles ? uu : u) * 4096u + 1024u * (j & 3) + 16u * lane));
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  uint32_t o0 = __builtin_nontemporal_load(off + t * 64u + lane), c0 = __builtin_nontemporal_load(cap + t * 64u + lane);
  wl(t);
  for (;;) {
#pragma unroll
    for (int j = 0; j < 8; j++) *reinterpret_cast<v4u *>(g_lds + buf + 1024u * j + 16u * lane) = wv[j];
    const uint32_t tn = t + 2 * nw;
    if (tn < ntiles) wl(tn);
    for (int h = 0; h < 2; h++) {
      const uint32_t tt = t + h * nw;
      if (tt < ntiles) {
        const uint32_t x = fake_decode<SPIN>(buf + 4096u * h + 64u * lane + (o0 & 15u), o0, c0);
        store_rec(rec, (uint64_t)tt * 64u + lane, x);
      }
    }
    if (tn >= ntiles) break;
    t = tn;
    o0 = __builtin_nontemporal_load(off + t * 64u + lane);
    c0 = __builtin_nontemporal_load(cap + t * 64u + lane);
  }
}

// LDS-DMA with NB buffers per wave (NB - 1 tiles in flight); a tile's DMA: 4 x 1 KiB data + 2
// descriptor loads = 6 VMEM instructions; the stores of a tile are issued after the next
// tile's DMA.  Wait for tile k at the top of iteration k: the VMEM instructions issued after
// tile k's DMA are (NB - 2) later tiles' DMAs and the stores of the NB - 1 preceding iterations.
template <int NB, int SPIN>
__global__ __launch_bounds__(256) void dma_k(const uint8_t *__restrict__ data, const uint32_t *__restrict__ off,
                                             const uint32_t *__restrict__ cap, v4u *rec, uint32_t ntiles) {
  constexpr uint32_t kSlot = 4096u + 512u;
  const uint32_t lane = threadIdx.x & 63u, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t nw = gridDim.x * 4u;
  const uint32_t base = wave * NB * kSlot;
  const uint32_t t0 = blockIdx.x * 4u + wave;
  if (t0 >= ntiles) return;
  const uint32_t mine = (ntiles - t0 + nw - 1u) / nw;  // tiles of this wave
  auto issue = [&](uint32_t k) {  // the wave's k-th tile into buffer k % NB
    const uint32_t u = t0 + k * nw, b = base + (k % NB) * kSlot;
#pragma unroll
    for (int j = 0; j < 4; j++) glds16(data + (uint64_t)u * 4096u + 1024u * j, 16u * lane, b + 1024u * j);
    glds4(off + u * 64u, 4u * lane, b + 4096u);
    glds4(cap + u * 64u, 4u * lane, b + 4096u + 256u);
  };
  for (uint32_t k = 0; k + 1 < NB && k < mine; k++) issue(k);
  for (uint32_t k = 0; k < mine; k++) {
    // tile k landed: later tiles' DMA in flight = min(NB - 2, mine - 1 - k); stores after it:
    // one per earlier iteration since tile k was issued (at most NB - 1; k of them exist)
    const uint32_t later = min((uint32_t)NB - 2u, mine - 1u - k);
    const uint32_t st = min((uint32_t)NB - 1u, k);
    if (later == (uint32_t)NB - 2u && st == (uint32_t)NB - 1u) vmwait<6 * (NB - 2) + 2 * (NB - 1)>();
    else vmwait<0>();
    if (k + NB - 1 < mine) issue(k + NB - 1);  // into the buffer tile k - 1 used
    const uint32_t b = base + (k % NB) * kSlot;
    const uint32_t o = *reinterpret_cast<const uint32_t *>(g_lds + b + 4096u + 4u * lane);
    const uint32_t c = *reinterpret_cast<const uint32_t *>(g_lds + b + 4096u + 256u + 4u * lane);
    const uint32_t x = fake_decode<SPIN>(b + 64u * lane + (o & 15u), o, c);
    store_rec(rec, (uint64_t)(t0 + k * nw) * 64u + lane, x);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // buffer k % NB read before reuse
  }
}

template <typename L>
static float timeit(L launch, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 300; r++) launch();  // clock settle
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

template <int SPIN>
static void run(int cus, const uint8_t *data, const uint32_t *off, const uint32_t *cap, v4u *rec, uint32_t ntiles,
                int reps) {
  const double bytes = (double)ntiles * 64.0 * (72.0 + 32.0);
  auto rep = [&](const char *nm, int wpc, float ms) {
    printf("RESULT spin=%d %-5s wpc=%d ms=%.4f TBps=%.3f\n", SPIN, nm, wpc, ms, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  for (int wpc : {1, 2, 3, 4}) {
    const dim3 g(cus * wpc);
    rep("reg", wpc, timeit([&] { hipLaunchKernelGGL(reg_k<SPIN>, g, dim3(256), 4 * 4096, 0, data, off, cap, rec, ntiles); }, reps));
    rep("reg2", wpc, timeit([&] { hipLaunchKernelGGL(reg2_k<SPIN>, g, dim3(256), 4 * 8192, 0, data, off, cap, rec, ntiles); }, reps));
    rep("dma2", wpc, timeit([&] { hipLaunchKernelGGL((dma_k<2, SPIN>), g, dim3(256), 4 * 2 * 4608, 0, data, off, cap, rec, ntiles); }, reps));
    if (wpc <= 2) {
      rep("dma3", wpc, timeit([&] { hipLaunchKernelGGL((dma_k<3, SPIN>), g, dim3(256), 4 * 3 * 4608, 0, data, off, cap, rec, ntiles); }, reps));
      rep("dma4", wpc, timeit([&] { hipLaunchKernelGGL((dma_k<4, SPIN>), g, dim3(256), 4 * 4 * 4608, 0, data, off, cap, rec, ntiles); }, reps));
    }
  }
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("stream_dma: %s %d CUs\n", prop.gcnArchName, cus);
  const uint32_t ntiles = 1u << 18;  // 2^24 packets of 64 B
  const uint64_t n = (uint64_t)ntiles * 64u;
  uint8_t *data = nullptr;
  uint32_t *off = nullptr, *cap = nullptr;
  v4u *rec = nullptr;
  CK(hipMalloc(&data, n * 64u));
  CK(hipMemset(data, 0x5a, n * 64u));
  CK(hipMalloc(&off, n * 4u));
  CK(hipMalloc(&cap, n * 4u));
  CK(hipMemset(off, 0, n * 4u));
  CK(hipMemset(cap, 0x40, n * 4u));
  CK(hipMalloc(&rec, n * 32u));
  run<0>(cus, data, off, cap, rec, ntiles, reps);
  run<64>(cus, data, off, cap, rec, ntiles, reps);
  run<128>(cus, data, off, cap, rec, ntiles, reps);
  run<192>(cus, data, off, cap, rec, ntiles, reps);
  CK(hipFree(data));
  CK(hipFree(off));
  CK(hipFree(cap));
  CK(hipFree(rec));
  return 0;
}
