// Tile-to-wave mapping probe (diagnostic, not product): the decode kernels hand wave w the
// 64-packet tiles w, w + W, w + 2W, ... (grid stride: at any moment the grid sweeps one region
// of ~W tiles together).  Does another mapping stream the same traffic faster on this part?
//   stride  : tile t -> wave t mod W, as the kernels do
//   block   : wave w takes a contiguous run of ceil(T/W) tiles (3072 sequential streams)
//   xcd     : grid stride over "XCD-local" wave numbers: consecutive tiles go to waves of the same
//             XCD (workgroups are dispatched round-robin over the 8 XCDs, so workgroup b runs on
//             XCD b mod 8; its waves take tile slots (b mod 8) * W/8 + b / 8 ...)
// Per tile: its read bytes as one contiguous run (16 B per lane, nt loads, rounds of 8 KiB in
// registers), then the results: SoA (u32 + u32 + 3 x u64 arrays, 64 lanes each) or AoS (two
// 16-B stores per lane).  Shapes: config 2 (64-B frames: 4,608 B per tile, 4 KiB rounds) and
// IMIX (23,190 B per tile).  hipcc --offload-arch=gfx950 -O3 -o tile_map tile_map.hip
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

enum Map { kStride = 0, kBlock = 1, kXcd = 2 };

template <int MAXC, int MAP, bool SOA>
__global__ __launch_bounds__(256) void tile_k(const v4u *__restrict__ in, uint32_t *st, uint32_t *cs,
                                              uint64_t *ly, uint64_t *nh, uint64_t *th, v4u *rec,
                                              uint32_t ntiles, uint32_t ctile) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  uint32_t w;  // this wave's slot in the mapping
  if (MAP == kXcd) {
    const uint32_t per = gridDim.x / 8u;  // workgroups per XCD (gridDim a multiple of 8)
    w = ((blockIdx.x & 7u) * per + (blockIdx.x >> 3)) * 4u + wave;
  } else {
    w = blockIdx.x * 4u + wave;
  }
  const uint32_t per_w = (ntiles + nw - 1) / nw;
  for (uint32_t k = 0;; k++) {
    uint32_t t;
    if (MAP == kBlock) {
      if (k >= per_w) break;
      t = w * per_w + k;
    } else {
      t = w + k * nw;
    }
    if (t >= ntiles) break;
    const v4u *p = in + (uint64_t)t * ctile;
    uint32_t x = 0;
    for (uint32_t c0 = 0; c0 < ctile; c0 += 64u * MAXC) {
      v4u v[MAXC];
#pragma unroll
      for (int j = 0; j < MAXC; j++) {
        const uint32_t c = c0 + 64u * j + lane;
        v[j] = c < ctile ? __builtin_nontemporal_load(p + c) : v4u{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int j = 0; j < MAXC; j++) x ^= v[j].x + v[j].y + v[j].z + v[j].w;
    }
    const uint64_t i = (uint64_t)t * 64u + lane;
    if (SOA) {
      __builtin_nontemporal_store(x, st + i);
      __builtin_nontemporal_store(x ^ 5u, cs + i);
      __builtin_nontemporal_store((uint64_t)x * 3u, ly + i);
      __builtin_nontemporal_store((uint64_t)x * 7u, nh + i);
      __builtin_nontemporal_store((uint64_t)x * 9u, th + i);
    } else {
      __builtin_nontemporal_store(v4u{x, x ^ 1u, x * 3u, 0u}, rec + 2 * i);
      __builtin_nontemporal_store(v4u{x * 5u, 0u, x * 7u, 0u}, rec + 2 * i + 1);
    }
  }
}

template <int MAXC, int MAP, bool SOA>
static float timeit(int wpc, int cus, const v4u *in, uint32_t *st, uint32_t *cs, uint64_t *ly, uint64_t *nh,
                    uint64_t *th, v4u *rec, uint32_t ntiles, uint32_t ctile, int reps) {
  const int g = cus * wpc;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 200; r++)  // clock settle
    hipLaunchKernelGGL((tile_k<MAXC, MAP, SOA>), dim3(g), dim3(256), 0, 0, in, st, cs, ly, nh, th, rec, ntiles, ctile);
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++)
    hipLaunchKernelGGL((tile_k<MAXC, MAP, SOA>), dim3(g), dim3(256), 0, 0, in, st, cs, ly, nh, th, rec, ntiles, ctile);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

template <int MAXC>
static void shape(const char *name, uint32_t ntiles, uint32_t tile_bytes, int cus, int reps) {
  const uint32_t ctile = (tile_bytes + 15u) / 16u;
  v4u *in = nullptr, *rec = nullptr;
  uint32_t *st = nullptr, *cs = nullptr;
  uint64_t *ly = nullptr, *nh = nullptr, *th = nullptr;
  const uint64_t n = (uint64_t)ntiles * 64u;
  CK(hipMalloc(&in, (size_t)ntiles * ctile * 16u));
  CK(hipMemset(in, 0x5a, (size_t)ntiles * ctile * 16u));
  CK(hipMalloc(&rec, n * 32));
  CK(hipMalloc(&st, n * 4));
  CK(hipMalloc(&cs, n * 4));
  CK(hipMalloc(&ly, n * 8));
  CK(hipMalloc(&nh, n * 8));
  CK(hipMalloc(&th, n * 8));
  const double bytes = (double)ntiles * (ctile * 16.0 + 2048.0);
  for (int wpc : {2, 3, 4}) {
    float t[6];
    t[0] = timeit<MAXC, kStride, false>(wpc, cus, in, st, cs, ly, nh, th, rec, ntiles, ctile, reps);
    t[1] = timeit<MAXC, kBlock, false>(wpc, cus, in, st, cs, ly, nh, th, rec, ntiles, ctile, reps);
    t[2] = timeit<MAXC, kXcd, false>(wpc, cus, in, st, cs, ly, nh, th, rec, ntiles, ctile, reps);
    t[3] = timeit<MAXC, kStride, true>(wpc, cus, in, st, cs, ly, nh, th, rec, ntiles, ctile, reps);
    t[4] = timeit<MAXC, kBlock, true>(wpc, cus, in, st, cs, ly, nh, th, rec, ntiles, ctile, reps);
    t[5] = timeit<MAXC, kXcd, true>(wpc, cus, in, st, cs, ly, nh, th, rec, ntiles, ctile, reps);
    const char *nm[6] = {"stride_aos", "block_aos", "xcd_aos", "stride_soa", "block_soa", "xcd_soa"};
    for (int k = 0; k < 6; k++)
      printf("RESULT %s wpc=%d %-10s ms=%.4f TBps=%.3f\n", name, wpc, nm[k], t[k], bytes / (t[k] * 1e-3) / 1e12);
  }
  CK(hipFree(in));
  CK(hipFree(rec));
  CK(hipFree(st));
  CK(hipFree(cs));
  CK(hipFree(ly));
  CK(hipFree(nh));
  CK(hipFree(th));
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("tile_map: %s %d CUs\n", prop.gcnArchName, cus);
  shape<5>("cfg2_64B", 1u << 18, 64u * 72u, cus, reps);   // 2^24 packets of 64 B + 8 B descriptors
  shape<8>("imix", 65536u, 23190u, cus, reps);            // 2^22 IMIX packets, 362.3 B read each
  return 0;
}
