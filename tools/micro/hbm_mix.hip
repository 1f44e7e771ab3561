// HBM ceiling probe (diagnostic, not product): what read+write mix rate can plain
// register-staged streaming reach on this box, next to hipMemcpy?  Kernels:
//   copy    : out[i] = in[i], 16 B per lane per access, U accesses in flight per lane
//   read    : sum of in[] (16 B per lane), one word written per workgroup
//   mix     : the decode kernel's traffic shape without the decode: per 64-packet tile read
//             64 x 72 B (packet bytes + descriptors) and write 64 x 32 B as five SoA stores
//   hipcc --offload-arch=gfx950 -O3 -o hbm_mix hbm_mix.hip && ./hbm_mix
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

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(const v4u *__restrict__ in, v4u *__restrict__ out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b + u * 256 < n) v[u] = NT ? __builtin_nontemporal_load(in + b + u * 256) : in[b + u * 256];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b + u * 256 < n) {
        if (NT) __builtin_nontemporal_store(v[u], out + b + u * 256);
        else out[b + u * 256] = v[u];
      }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const v4u *__restrict__ in, uint32_t *out, uint64_t n) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  uint32_t acc = 0;
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n; b += stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++)
      if (b + u * 256 < n) v[u] = __builtin_nontemporal_load(in + b + u * 256);
#pragma unroll
    for (int u = 0; u < U; u++) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// One wave per 64-packet tile: 4.5 KiB of packet bytes + descriptors read as 16-B lanes
// (288 x 16 B), then status/layers/net/tp/csum written for 64 packets.
template <int T>
__global__ __launch_bounds__(256) void mix_k(const v4u *__restrict__ in, uint32_t *st, uint64_t *ly,
                                            uint64_t *nh, uint64_t *th, uint32_t *cs, uint32_t ntiles) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4;
  for (uint32_t t0 = blockIdx.x * 4 + wave; t0 < ntiles; t0 += nw * T) {
    v4u v[T][5];
#pragma unroll
    for (int t = 0; t < T; t++) {
      const uint32_t tile = t0 + t * nw;
      if (tile < ntiles) {
        const v4u *p = in + (uint64_t)tile * 288;
#pragma unroll
        for (int k = 0; k < 4; k++) v[t][k] = __builtin_nontemporal_load(p + k * 64 + lane);
        v[t][4] = lane < 32 ? __builtin_nontemporal_load(p + 256 + lane) : v4u{0u, 0u, 0u, 0u};
      }
    }
#pragma unroll
    for (int t = 0; t < T; t++) {
      const uint32_t tile = t0 + t * nw;
      if (tile < ntiles) {
        uint32_t x = 0;
#pragma unroll
        for (int k = 0; k < 5; k++) x ^= v[t][k].x + v[t][k].y + v[t][k].z + v[t][k].w;
        const uint64_t i = (uint64_t)tile * 64 + lane;
        __builtin_nontemporal_store(x, st + i);
        __builtin_nontemporal_store((uint64_t)x * 3, ly + i);
        __builtin_nontemporal_store((uint64_t)x * 5, nh + i);
        __builtin_nontemporal_store((uint64_t)x * 7, th + i);
        __builtin_nontemporal_store(x ^ 1u, cs + i);
      }
    }
  }
}

// mix through LDS with register prefetch: the next tile's 4.5 KiB is loaded into VGPRs while
// the current tile (already copied to the wave's LDS slot) is read back at a per-lane packet
// offset and its records stored.  The shape of a register-staged decode loop.
__global__ __launch_bounds__(256) void mix_lds_k(const v4u *__restrict__ in, uint32_t *st, uint64_t *ly,
                                                uint64_t *nh, uint64_t *th, uint32_t *cs, uint32_t ntiles,
                                                int work) {
  __shared__ v4u lds[4][288];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4;
  uint32_t t = blockIdx.x * 4 + wave;
  v4u v[5];
  auto load = [&](uint32_t tile) {
    const v4u *p = in + (uint64_t)tile * 288;
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = __builtin_nontemporal_load(p + k * 64 + lane);
    v[4] = lane < 32 ? __builtin_nontemporal_load(p + 256 + lane) : v4u{0u, 0u, 0u, 0u};
  };
  if (t < ntiles) load(t);
  for (; t < ntiles; t += nw) {
#pragma unroll
    for (int k = 0; k < 4; k++) lds[wave][k * 64 + lane] = v[k];
    if (lane < 32) lds[wave][256 + lane] = v[4];
    if (t + nw < ntiles) load(t + nw);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS copy landed (own wave only)
    const v4u q = lds[wave][(lane * 4 + 3) % 288];
    uint32_t x = q.x ^ q.y ^ q.z ^ q.w;
    for (int r = 0; r < work; r++) x = x * 0x9E3779B1u + (x >> 7);
    const uint64_t i = (uint64_t)t * 64 + lane;
    __builtin_nontemporal_store(x, st + i);
    __builtin_nontemporal_store((uint64_t)x * 3, ly + i);
    __builtin_nontemporal_store((uint64_t)x * 5, nh + i);
    __builtin_nontemporal_store((uint64_t)x * 7, th + i);
    __builtin_nontemporal_store(x ^ 1u, cs + i);
  }
}

// The same loop with the results written as MODE: 0 five SoA streams (the decode's layout),
// 1 six SoA streams (+ a u32 hdr_off), 2 one AoS stream of 32-B records (two 16-B stores per
// lane), 3 AoS 32-B records staged through LDS so each store instruction writes 1 KiB
// contiguous (lane l writes bytes 16 l of the wave's 2 KiB of records).
template <int MODE>
__global__ __launch_bounds__(256) void mix_out_k(const v4u *__restrict__ in, uint32_t *st, uint64_t *ly,
                                                uint64_t *nh, uint64_t *th, uint32_t *cs, uint32_t *ho,
                                                v4u *rec, uint32_t ntiles, int work) {
  __shared__ v4u lds[4][288];
  __shared__ v4u orec[4][128];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4;
  uint32_t t = blockIdx.x * 4 + wave;
  v4u v[5];
  auto load = [&](uint32_t tile) {
    const v4u *p = in + (uint64_t)tile * 288;
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = __builtin_nontemporal_load(p + k * 64 + lane);
    v[4] = lane < 32 ? __builtin_nontemporal_load(p + 256 + lane) : v4u{0u, 0u, 0u, 0u};
  };
  if (t < ntiles) load(t);
  for (; t < ntiles; t += nw) {
#pragma unroll
    for (int k = 0; k < 4; k++) lds[wave][k * 64 + lane] = v[k];
    if (lane < 32) lds[wave][256 + lane] = v[4];
    if (t + nw < ntiles) load(t + nw);
    __builtin_amdgcn_s_waitcnt(0xc07f);
    const v4u q = lds[wave][(lane * 4 + 3) % 288];
    uint32_t x = q.x ^ q.y ^ q.z ^ q.w;
    for (int r = 0; r < work; r++) x = x * 0x9E3779B1u + (x >> 7);
    const uint64_t i = (uint64_t)t * 64 + lane;
    if (MODE <= 1) {
      __builtin_nontemporal_store(x, st + i);
      __builtin_nontemporal_store((uint64_t)x * 3, ly + i);
      __builtin_nontemporal_store((uint64_t)x * 5, nh + i);
      __builtin_nontemporal_store((uint64_t)x * 7, th + i);
      __builtin_nontemporal_store(x ^ 1u, cs + i);
      if (MODE == 1) __builtin_nontemporal_store(x ^ 3u, ho + i);
    } else if (MODE == 2) {
      __builtin_nontemporal_store(v4u{x, x ^ 1u, x * 3u, 0u}, rec + 2 * i);
      __builtin_nontemporal_store(v4u{x * 5u, 0u, x * 7u, 0u}, rec + 2 * i + 1);
    } else {
      orec[wave][2 * lane] = v4u{x, x ^ 1u, x * 3u, 0u};
      orec[wave][2 * lane + 1] = v4u{x * 5u, 0u, x * 7u, 0u};
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_nontemporal_store(orec[wave][lane], rec + (uint64_t)t * 128 + lane);
      __builtin_nontemporal_store(orec[wave][64 + lane], rec + (uint64_t)t * 128 + 64 + lane);
    }
  }
}

template <class F>
static float time_ms(F f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; r++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  int cus = 256;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  cus = prop.multiProcessorCount;
  const uint64_t bytes = 1ull << 30, n = bytes / 16;
  v4u *a, *b;
  const uint64_t abytes = 288ull * 16 * (1u << 18);  // the mix reads 2^18 tiles x 4.5 KiB
  CK(hipMalloc(&a, abytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, abytes));
  CK(hipMemset(b, 2, bytes));
  float ms = time_ms([&] { CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice)); });
  printf("hipMemcpy D2D 1 GiB            %.4f ms  %6.0f GB/s (r+w)\n", ms, 2 * bytes / ms / 1e6);
  for (int wpc : {2, 4, 8, 16}) {
    const int g = cus * wpc;
    ms = time_ms([&] { hipLaunchKernelGGL((copy_k<4, false>), dim3(g), dim3(256), 0, 0, a, b, n); });
    printf("copy U4      wg/cu %2d          %.4f ms  %6.0f GB/s (r+w)\n", wpc, ms, 2 * bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(g), dim3(256), 0, 0, a, b, n); });
    printf("copy U4 nt   wg/cu %2d          %.4f ms  %6.0f GB/s (r+w)\n", wpc, ms, 2 * bytes / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((read_k<4>), dim3(g), dim3(256), 0, 0, a, (uint32_t *)b, n); });
    printf("read U4 nt   wg/cu %2d          %.4f ms  %6.0f GB/s (r)\n", wpc, ms, bytes / ms / 1e6);
  }
  // decode-shaped mix: 2^24 packets, 72 B read + 32 B written each
  const uint32_t ntiles = 1u << 18;
  uint32_t *st, *cs;
  uint64_t *ly, *nh, *th;
  CK(hipMalloc(&st, 4ull << 24));
  CK(hipMalloc(&cs, 4ull << 24));
  CK(hipMalloc(&ly, 8ull << 24));
  CK(hipMalloc(&nh, 8ull << 24));
  CK(hipMalloc(&th, 8ull << 24));
  const double rd = 72.0 * (1 << 24), wr = 32.0 * (1 << 24);
  for (int wpc : {2, 4, 8}) {
    const int g = cus * wpc;
    ms = time_ms([&] { hipLaunchKernelGGL((mix_k<1>), dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ntiles); });
    printf("mix72/32 T1  wg/cu %2d          %.4f ms  %6.0f GB/s (r+w)  read %.0f\n", wpc, ms, (rd + wr) / ms / 1e6, rd / ms / 1e6);
    ms = time_ms([&] { hipLaunchKernelGGL((mix_k<2>), dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ntiles); });
    printf("mix72/32 T2  wg/cu %2d          %.4f ms  %6.0f GB/s (r+w)  read %.0f\n", wpc, ms, (rd + wr) / ms / 1e6, rd / ms / 1e6);
  }
  for (int wpc : {2, 3, 4}) {
    for (int work : {0, 64, 128}) {
      const int g = cus * wpc;
      ms = time_ms([&] { hipLaunchKernelGGL(mix_lds_k, dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ntiles, work); });
      printf("mixLDS work %3d wg/cu %2d       %.4f ms  %6.0f GB/s (r+w)  read %.0f\n", work, wpc, ms, (rd + wr) / ms / 1e6, rd / ms / 1e6);
    }
  }
  uint32_t *ho;
  v4u *rec;
  CK(hipMalloc(&ho, 4ull << 24));
  CK(hipMalloc(&rec, 32ull << 24));
  const char *names[4] = {"SoA5", "SoA6", "AoS32", "AoS32lds"};
  for (int wpc : {3, 4}) {
    for (int work : {0, 64, 128}) {
      for (int rep = 0; rep < 2; rep++) {
        for (int mode = 0; mode < 4; mode++) {
          const int g = cus * wpc;
          auto f = [&] {
            switch (mode) {
              case 0: hipLaunchKernelGGL(mix_out_k<0>, dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ho, rec, ntiles, work); break;
              case 1: hipLaunchKernelGGL(mix_out_k<1>, dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ho, rec, ntiles, work); break;
              case 2: hipLaunchKernelGGL(mix_out_k<2>, dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ho, rec, ntiles, work); break;
              default: hipLaunchKernelGGL(mix_out_k<3>, dim3(g), dim3(256), 0, 0, a, st, ly, nh, th, cs, ho, rec, ntiles, work); break;
            }
          };
          ms = time_ms(f);
          const double w = mode == 1 ? 36.0 * (1 << 24) : wr;
          printf("out %-8s work %3d wg/cu %d   %.4f ms  %6.0f GB/s (r+w)\n", names[mode], work, wpc, ms, (rd + w) / ms / 1e6);
        }
      }
    }
  }
  return 0;
}
