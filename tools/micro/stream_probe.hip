// Streaming-skeleton probe: how fast can a wave-per-tile LDS-DMA stream with a result
// write per packet run on this chip, as a function of ring depth, slot size, waves per CU
// and tile order?  No decode: each lane reads one 16-B chunk of its packet from LDS and
// writes a 32-B record (status u32, three u64, csum u32 as five SoA stores), like the
// decode kernel's skeleton.  Standalone (no torch):
//   hipcc --offload-arch=gfx950 -O3 -o stream_probe stream_probe.hip && ./stream_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

extern __shared__ __attribute__((aligned(16))) uint8_t g_lds[];

__device__ __forceinline__ void glds16(const uint8_t *gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void glds4(const void *gbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dword %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(gbase), "s"(lds)
      : "memory");
}
template <int N>
__device__ __forceinline__ void wait_le() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt vmcnt(min(n, 63)): everything but the n most recent VMEM instructions retired
__device__ __forceinline__ void wait_vm(uint32_t n) {
  switch (n) {
#define W(k) case k: wait_le<k>(); break;
    W(0) W(1) W(2) W(3) W(4) W(5) W(6) W(7) W(8) W(9) W(10) W(11) W(12) W(13) W(14) W(15)
    W(16) W(17) W(18) W(19) W(20) W(21) W(22) W(23) W(24) W(25) W(26) W(27) W(28) W(29) W(30)
    W(31) W(32) W(33) W(34) W(35) W(36) W(37) W(38) W(39) W(40) W(41) W(42) W(43) W(44) W(45)
    W(46) W(47) W(48) W(49) W(50) W(51) W(52) W(53) W(54) W(55) W(56) W(57) W(58) W(59) W(60)
    W(61) W(62)
#undef W
    default: wait_le<63>(); break;
  }
}

struct P {
  const uint8_t *data;
  uint32_t *st;
  uint64_t *l, *nh, *th;
  uint32_t *cs;
  uint32_t ntiles;
  uint32_t tile_bytes;  // bytes per tile (64 packets)
  uint32_t store;       // 1: write the 32-B records
  uint32_t work;        // dependent VALU rounds per tile (x8 chains)
  uint32_t desc;        // 1: descriptor DMA per tile (2 x glds4, two tiles ahead) + LDS read
  const uint32_t *off, *cap;
};

// S: slot bytes (a tile is S bytes here); R: ring slots per wave; WAVES per workgroup.
// ORDER 0: grid-stride tiles (t, t + W, ...); 1: contiguous tile range per wave.
template <int S, int R, int WAVES, int ORDER>
__global__ __launch_bounds__(64 * WAVES) void stream(P p) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t ring = wave * (S * R);
  const uint32_t nw = gridDim.x * WAVES;
  const uint32_t gw = blockIdx.x * WAVES + wave;
  uint32_t t0, tstep, tcount;
  if (ORDER == 0) {
    t0 = gw;
    tstep = nw;
    tcount = gw < p.ntiles ? (p.ntiles - gw + nw - 1) / nw : 0;
  } else {
    const uint32_t per = p.ntiles / nw, extra = p.ntiles % nw;
    t0 = gw * per + min(gw, extra);
    tcount = per + (gw < extra ? 1 : 0);
    tstep = 1;
  }
  if (tcount == 0) return;
  const uint32_t dsl = S * R * WAVES + wave * 2048u;  // 4 desc slots of 512 B
  uint32_t issued = 0;  // VMEM instructions issued by this wave
  uint32_t mark[R];     // `issued` right after each slot's DMA (rotating)
  auto issue = [&](uint32_t k) {  // tile number k of this wave -> slot k % R
    const uint32_t t = t0 + k * tstep;
    const uint32_t lds = ring + (k % R) * S;
    if (p.desc) {
      const uint32_t td = t0 + (k + 2) * tstep;
      if (k + 2 < tcount) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        glds4(p.off + td * 64u, 4u * lane, dsl + ((k + 2) & 3u) * 512u);
        glds4(p.cap + td * 64u, 4u * lane, dsl + ((k + 2) & 3u) * 512u + 256u);
        issued += 2;
      }
      // plan: read this window's descriptors (landed two issues ago)
      const uint32_t o = *reinterpret_cast<const uint32_t *>(g_lds + dsl + (k & 3u) * 512u + 4u * lane);
      const uint32_t b0 = __builtin_amdgcn_readfirstlane(o);
      if (b0 == 0xFFFFFFFFu) return;
    }
#pragma unroll
    for (uint32_t c = 0; c < (uint32_t)S; c += 1024u)
      glds16(p.data + (uint64_t)t * p.tile_bytes + c, 16u * lane, lds + c);
    issued += S / 1024;
  };
#pragma unroll
  for (int k = 0; k < R - 1; k++) {
    if ((uint32_t)k < tcount) issue(k);
    mark[k] = issued;
  }
  uint32_t acc = 0;
  for (uint32_t k = 0; k < tcount; k++) {
    wait_vm(issued - mark[0]);
#pragma unroll
    for (int r = 0; r < R - 1; r++) mark[r] = mark[r + 1];
    if (k + R - 1 < tcount) issue(k + R - 1);
    mark[R - 1] = issued;
    // consume: each lane one 16-B chunk of its packet
    const uint32_t pk = (S / 64) * lane;
    const uint4 q = *reinterpret_cast<const uint4 *>(g_lds + ring + (k % R) * S + pk);
    acc = q.x ^ q.y ^ q.z ^ q.w ^ (acc * 3);
    {
      uint32_t c[8] = {q.x, q.y, q.z, q.w, q.x + 1, q.y + 1, q.z + 1, q.w + 1};
      for (uint32_t r = 0; r < p.work; r++) {
#pragma unroll
        for (int j = 0; j < 8; j++) c[j] = __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, c[j]), __builtin_bit_cast(u16x2, 0x00010001u), c[j], false);
      }
      acc += c[0] ^ c[1] ^ c[2] ^ c[3] ^ c[4] ^ c[5] ^ c[6] ^ c[7];
    }
    if (p.store) {
      const uint32_t i = (t0 + k * tstep) * 64u + lane;
      p.st[i] = acc;
      p.l[i] = acc * 5ull;
      p.nh[i] = acc * 7ull;
      p.th[i] = acc * 9ull;
      p.cs[i] = acc + 1;
      issued += 5;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int S, int R, int WAVES, int ORDER>
static void run(const P &p, int cus, int wg_per_cu, const char *name) {
  const size_t lds = (size_t)S * R * WAVES + 2048 * WAVES;
  if (lds * wg_per_cu > 160 * 1024) return;
  // pad LDS so exactly wg_per_cu workgroups fit on a CU
  size_t alloc = (160 * 1024) / wg_per_cu;
  if (alloc > 160 * 1024) alloc = 160 * 1024;
  alloc &= ~(size_t)1023;
  if (alloc < lds) alloc = lds;
  const int blocks = cus * wg_per_cu;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; w++) hipLaunchKernelGGL((stream<S, R, WAVES, ORDER>), dim3(blocks), dim3(64 * WAVES), alloc, 0, p);
  CK(hipEventRecord(a));
  const int iters = 20;
  for (int w = 0; w < iters; w++)
    hipLaunchKernelGGL((stream<S, R, WAVES, ORDER>), dim3(blocks), dim3(64 * WAVES), alloc, 0, p);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  ms /= iters;
  const double rb = (double)p.ntiles * p.tile_bytes;
  const double wb = p.store ? (double)p.ntiles * 64 * 32 : 0;
  printf("%-24s S=%5d R=%d w=%d wg/cu=%d ord=%d st=%d work=%d desc=%d  %.4f ms  read %.0f GB/s  total %.0f GB/s\n",
         name, S, R, WAVES, wg_per_cu, ORDER, p.store, p.work, p.desc, ms, rb / ms / 1e6, (rb + wb) / ms / 1e6);
  fflush(stdout);
}

int main(int argc, char **argv) {
  int dev = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, dev));
  const int cus = prop.multiProcessorCount;
  const uint32_t npk = 1u << 24;  // 64-B packets
  P p{};
  uint8_t *d;
  CK(hipMalloc(&d, (size_t)npk * 64 + 8192));
  CK(hipMemset(d, 0x5a, (size_t)npk * 64 + 8192));
  p.data = d;
  CK(hipMalloc(&p.st, (size_t)npk * 4));
  CK(hipMalloc(&p.l, (size_t)npk * 8));
  CK(hipMalloc(&p.nh, (size_t)npk * 8));
  CK(hipMalloc(&p.th, (size_t)npk * 8));
  CK(hipMalloc(&p.cs, (size_t)npk * 4));
  // copy reference
  {
    uint8_t *d2;
    CK(hipMalloc(&d2, (size_t)npk * 64));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int w = 0; w < 3; w++) CK(hipMemcpyAsync(d2, d, (size_t)npk * 64, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(a));
    for (int w = 0; w < 10; w++) CK(hipMemcpyAsync(d2, d, (size_t)npk * 64, hipMemcpyDeviceToDevice));
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 10;
    printf("hipMemcpy D2D 1 GiB: %.4f ms  %.0f GB/s (read+write)\n", ms, 2.0 * npk * 64 / ms / 1e6);
    CK(hipFree(d2));
  }
  uint32_t *off, *cap;
  CK(hipMalloc(&off, (size_t)npk * 4));
  CK(hipMalloc(&cap, (size_t)npk * 4));
  CK(hipMemset(off, 0, (size_t)npk * 4));
  CK(hipMemset(cap, 0, (size_t)npk * 4));
  p.off = off;
  p.cap = cap;
  p.store = 1;
  p.tile_bytes = 4096;
  p.ntiles = npk / 64;
  for (int desc = 0; desc <= 1; desc++) {
    p.desc = desc;
    for (int work : {0, 16, 32, 64}) {
      p.work = work;
      run<4096, 2, 4, 0>(p, cus, 3, "R2");
      run<4096, 3, 4, 0>(p, cus, 3, "R3");
      run<4096, 4, 4, 0>(p, cus, 2, "R4");
      run<4096, 3, 4, 0>(p, cus, 2, "R3 wg2");
      run<4096, 3, 8, 0>(p, cus, 1, "R3 8w");
      run<4096, 4, 8, 0>(p, cus, 1, "R4 8w");
      run<4096, 2, 8, 0>(p, cus, 2, "R2 8w");
    }
  }
  return 0;
}
