// Descriptor-load probe (diagnostic, not product): does the way a tile's 64 offsets and 64
// caplens are loaded (two u32 arrays, the gpd_batch layout) change the streaming rate of the
// decode's traffic shape?  Each wave: per 64-packet tile read 4 KiB of packet bytes as 16 B per
// lane (4 loads) through one LDS buffer with register prefetch (rs_kernel's loop shape), read
// the tile's descriptors, store five SoA records per packet.  Variants:
//   D0  no descriptors (the bytes alone: 64 B per packet)
//   D1  descriptors as two u32 loads per lane per tile, two tiles ahead (rs_kernel today)
//   D4  four consecutive tiles per wave step; their 256 offsets and 256 caplens as one
//       16-B load per lane each, handed to the packet lanes through LDS
//   hipcc --offload-arch=gfx950 -O3 -o desc_probe desc_probe.hip && ./desc_probe
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

struct Args {
  const v4u *data;
  const uint32_t *off, *cap;
  uint32_t *st, *cs;
  uint64_t *ly, *nh, *th;
  uint32_t ntiles;
};

__device__ __forceinline__ void store5(const Args &A, uint64_t i, uint32_t x) {
  __builtin_nontemporal_store(x, A.st + i);
  __builtin_nontemporal_store((uint64_t)x * 3, A.ly + i);
  __builtin_nontemporal_store((uint64_t)x * 5, A.nh + i);
  __builtin_nontemporal_store((uint64_t)x * 7, A.th + i);
  __builtin_nontemporal_store(x ^ 1u, A.cs + i);
}

template <int D>
__global__ __launch_bounds__(256) void probe(Args A) {
  __shared__ v4u lds[4][256];
  __shared__ uint32_t dl[4][2][256];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4;
  constexpr uint32_t Q = D == 4 ? 4 : 1;  // tiles per wave step
  uint32_t t = (blockIdx.x * 4 + wave) * Q;
  v4u v[4];
  auto load = [&](uint32_t tile) {
    const v4u *p = A.data + (uint64_t)tile * 256;
#pragma unroll
    for (int k = 0; k < 4; k++) v[k] = __builtin_nontemporal_load(p + k * 64 + lane);
  };
  uint32_t o1 = 0, c1 = 0, o2 = 0, c2 = 0;
  v4u od, cd;
  if (D == 1) {
    if (t < A.ntiles) { o1 = __builtin_nontemporal_load(A.off + t * 64 + lane); c1 = __builtin_nontemporal_load(A.cap + t * 64 + lane); }
    if (t + nw < A.ntiles) { o2 = __builtin_nontemporal_load(A.off + (t + nw) * 64 + lane); c2 = __builtin_nontemporal_load(A.cap + (t + nw) * 64 + lane); }
  }
  if (D == 4 && t < A.ntiles) {
    od = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(A.off + t * 64) + lane);
    cd = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(A.cap + t * 64) + lane);
  }
  if (t < A.ntiles) load(t);
  for (; t < A.ntiles; t += nw * Q) {
    if (D == 4) {  // the step's descriptors into LDS, the next step's in flight
      reinterpret_cast<v4u *>(dl[wave][0])[lane] = od;
      reinterpret_cast<v4u *>(dl[wave][1])[lane] = cd;
      const uint32_t tn = t + nw * Q;
      if (tn < A.ntiles) {
        od = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(A.off + tn * 64) + lane);
        cd = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(A.cap + tn * 64) + lane);
      }
    }
#pragma unroll
    for (uint32_t q = 0; q < Q; q++) {
      const uint32_t tile = t + q;
#pragma unroll
      for (int k = 0; k < 4; k++) lds[wave][k * 64 + lane] = v[k];
      const uint32_t nt = q + 1 < Q ? tile + 1 : t + nw * Q;  // the next tile this wave reads
      if (nt < A.ntiles) load(nt);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      uint32_t off = 0, cap = 0;
      if (D == 1) {
        off = o1, cap = c1;
        o1 = o2, c1 = c2;
        const uint32_t t2 = tile + 2 * nw;
        if (t2 < A.ntiles) { o2 = __builtin_nontemporal_load(A.off + t2 * 64 + lane); c2 = __builtin_nontemporal_load(A.cap + t2 * 64 + lane); }
      } else if (D == 4) {
        off = dl[wave][0][q * 64 + lane];
        cap = dl[wave][1][q * 64 + lane];
      }
      const v4u x4 = lds[wave][(lane * 4 + (off & 3) + (cap & 1)) & 255];
      const uint32_t x = x4.x ^ x4.y ^ x4.z ^ x4.w ^ off ^ cap;
      store5(A, (uint64_t)tile * 64 + lane, x);
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
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint32_t ntiles = 1u << 18;  // 2^24 packets of 64 B
  Args A;
  A.ntiles = ntiles;
  CK(hipMalloc((void **)&A.data, 4096ull * ntiles));
  CK(hipMalloc((void **)&A.off, 256ull * ntiles));
  CK(hipMalloc((void **)&A.cap, 256ull * ntiles));
  CK(hipMemset((void *)A.data, 1, 4096ull * ntiles));
  CK(hipMemset((void *)A.off, 0, 256ull * ntiles));
  CK(hipMemset((void *)A.cap, 0, 256ull * ntiles));
  CK(hipMalloc((void **)&A.st, 4ull << 24));
  CK(hipMalloc((void **)&A.cs, 4ull << 24));
  CK(hipMalloc((void **)&A.ly, 8ull << 24));
  CK(hipMalloc((void **)&A.nh, 8ull << 24));
  CK(hipMalloc((void **)&A.th, 8ull << 24));
  for (int rep = 0; rep < 2; rep++) {
    for (int wpc : {2, 4}) {
      const int g = cus * wpc;
      float ms0 = time_ms([&] { hipLaunchKernelGGL(probe<0>, dim3(g), dim3(256), 0, 0, A); });
      float ms1 = time_ms([&] { hipLaunchKernelGGL(probe<1>, dim3(g), dim3(256), 0, 0, A); });
      float ms4 = time_ms([&] { hipLaunchKernelGGL(probe<4>, dim3(g), dim3(256), 0, 0, A); });
      const double b0 = (64.0 + 32.0) * (1 << 24), b1 = (72.0 + 32.0) * (1 << 24);
      printf("wg/cu %d  D0 %.4f ms %5.0f GB/s   D1 %.4f ms %5.0f GB/s   D4 %.4f ms %5.0f GB/s\n", wpc, ms0,
             b0 / ms0 / 1e6, ms1, b1 / ms1 / 1e6, ms4, b1 / ms4 / 1e6);
    }
  }
  return 0;
}
