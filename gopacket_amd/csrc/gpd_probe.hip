// gpd_probe.hip — the attainable-bandwidth probe printed beside each roofline in bench.py.
//
// Diagnostic only (libgpd_probe.so, not part of the C-ABI in include/): how fast does plain
// register-staged streaming move the SAME traffic shape as a decode launch on this box — per
// 64-packet tile, the tile's algorithmic read bytes (packet bytes + descriptors) as one
// contiguous run loaded 16 B per lane, and its 64 x 32-B result records written as two
// 16-B nontemporal stores per lane — with no decode and no packet boundaries?  A decode
// kernel's `frac` against HBM peak reads against this figure: the gap between the two is the
// decode's and the window planner's cost, the gap between this and 1.0 is the part's.
// (tools/micro/hbm_mix.hip is the sweep this was taken from; its "mix72/32" row.)
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

constexpr uint32_t kMaxTileBytes = 1u << 20;  // read bytes per tile accepted

// One wave per 64-packet tile (grid stride).  ctile: the tile's 16-B read chunks; lane l loads
// chunks l, l + 64, ... of the tile, MAXC per lane in flight together (rounds of them for long
// tiles), folds them, then stores the tile's records.
template <int MAXC, bool COMMIT = false>
__global__ __launch_bounds__(256) void probe_k(const v4u *__restrict__ in, v4u *__restrict__ rec,
                                               uint32_t ntiles, uint32_t ctile) {
  extern __shared__ v4u lds[];  // COMMIT: each round's chunks are copied to the wave's LDS first
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  for (uint32_t t = blockIdx.x * 4u + wave; t < ntiles; t += nw) {
    const v4u *p = in + (uint64_t)t * ctile;
    uint32_t x = 0;
    for (uint32_t c0 = 0; c0 < ctile; c0 += 64u * MAXC) {
      v4u v[MAXC];
#pragma unroll
      for (int j = 0; j < MAXC; j++) {
        const uint32_t c = c0 + 64u * j + lane;
        v[j] = c < ctile ? __builtin_nontemporal_load(p + c) : v4u{0u, 0u, 0u, 0u};
      }
      if (COMMIT) {
#pragma unroll
        for (int j = 0; j < MAXC; j++) lds[(wave * MAXC + j) * 64 + lane] = v[j];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        const v4u q = lds[(wave * MAXC) * 64 + ((lane * 5 + 3) & 63)];
        x ^= q.x + q.y;
      }
#pragma unroll
      for (int j = 0; j < MAXC; j++) x ^= v[j].x + v[j].y + v[j].z + v[j].w;
    }
    const uint64_t i = (uint64_t)t * 64u + lane;
    __builtin_nontemporal_store(v4u{x, x ^ 1u, x * 3u, 0u}, rec + 2 * i);
    __builtin_nontemporal_store(v4u{x * 5u, 0u, x * 7u, 0u}, rec + 2 * i + 1);
  }
}

// The same with the results as the five SoA arrays of gpd_result (status u32, layers u64,
// net_hash u64, tp_hash u64, csum u32: the same 32 B per packet as five coalesced stores per
// tile), the form BASELINE config 3 asks for.
template <int MAXC>
__global__ __launch_bounds__(256) void probe_soa_k(const v4u *__restrict__ in, uint8_t *__restrict__ rec,
                                                   uint32_t ntiles, uint32_t ctile) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  const uint64_t n = (uint64_t)ntiles * 64u;
  uint32_t *st = reinterpret_cast<uint32_t *>(rec), *cs = st + n;
  uint64_t *ly = reinterpret_cast<uint64_t *>(cs + n), *nh = ly + n, *th = nh + n;
  for (uint32_t t = blockIdx.x * 4u + wave; t < ntiles; t += nw) {
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
    __builtin_nontemporal_store(x, st + i);
    __builtin_nontemporal_store((uint64_t)x * 3u, ly + i);
    __builtin_nontemporal_store((uint64_t)x * 5u, nh + i);
    __builtin_nontemporal_store((uint64_t)x * 7u, th + i);
    __builtin_nontemporal_store(x ^ 9u, cs + i);
  }
}

// Reads only (the north star's "HBM-read roofline" measured on the box): the same loads, no
// result stores (one store per wave that never fires keeps the loads live).
template <int MAXC>
__global__ __launch_bounds__(256) void probe_read_k(const v4u *__restrict__ in, v4u *__restrict__ rec,
                                                    uint32_t ntiles, uint32_t ctile) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  uint32_t x = 0;
  for (uint32_t t = blockIdx.x * 4u + wave; t < ntiles; t += nw) {
    const v4u *p = in + (uint64_t)t * ctile;
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
  }
  if (x == 0x9E3779B9u) rec[blockIdx.x * 256u + threadIdx.x] = v4u{x, 0u, 0u, 0u};
}

}  // namespace

extern "C" {

// Streams ntiles tiles of read_bytes_per_tile (rounded up to 16, at most 1 MiB) and 2 KiB of
// records each, at 2 and 4 workgroups per CU, `reps` timed launches after `warm_ms` of untimed
// ones; *best_ms is the fastest configuration's mean launch time.  0 on success, else the HIP
// error code.  Allocates and frees its own buffers.
int gpd_probe_stream2(int device, uint32_t ntiles, uint32_t read_bytes_per_tile, int reps, float warm_ms,
                      int soa, float *best_ms);

int gpd_probe_stream(int device, uint32_t ntiles, uint32_t read_bytes_per_tile, int reps, float warm_ms,
                     float *best_ms) {
  return gpd_probe_stream2(device, ntiles, read_bytes_per_tile, reps, warm_ms, 0, best_ms);
}

// gpd_probe_stream with the results stored as two 16-B records per lane (soa = 0, the gpd_record
// form), as the five SoA arrays (soa = 1), or not at all (soa = 2: the read-only ceiling).
int gpd_probe_stream2(int device, uint32_t ntiles, uint32_t read_bytes_per_tile, int reps, float warm_ms,
                      int soa, float *best_ms) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  const uint32_t ctile = (read_bytes_per_tile + 15u) / 16u;
  if (ctile == 0 || ctile > kMaxTileBytes / 16u || ntiles == 0 || reps <= 0) return (int)hipErrorInvalidValue;
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return (int)e;
  v4u *in = nullptr, *rec = nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  float best = 0.0f;
  if ((e = hipMalloc(&in, (size_t)ntiles * ctile * 16u)) != hipSuccess) goto done;
  if ((e = hipMalloc(&rec, (size_t)ntiles * 2048u)) != hipSuccess) goto done;
  if ((e = hipMemset(in, 0x5a, (size_t)ntiles * ctile * 16u)) != hipSuccess) goto done;
  if ((e = hipEventCreate(&a)) != hipSuccess || (e = hipEventCreate(&b)) != hipSuccess) goto done;
  for (int wpc : {2, 4}) {
    const uint32_t g = (uint32_t)prop.multiProcessorCount * (uint32_t)wpc;
    const uint32_t pl = (ctile + 63u) / 64u;  // chunks per lane per tile
    auto launch = [&] {  // a 64-B-frame tile (4.5 KiB) in one round; longer tiles in rounds of 8 KiB
      if (soa == 2) {  // reads only
        if (pl <= 5u) hipLaunchKernelGGL(probe_read_k<5>, dim3(g), dim3(256), 0, 0, in, rec, ntiles, ctile);
        else hipLaunchKernelGGL(probe_read_k<8>, dim3(g), dim3(256), 0, 0, in, rec, ntiles, ctile);
      } else if (soa) {
        uint8_t *r8 = reinterpret_cast<uint8_t *>(rec);
        if (pl <= 5u) hipLaunchKernelGGL(probe_soa_k<5>, dim3(g), dim3(256), 0, 0, in, r8, ntiles, ctile);
        else hipLaunchKernelGGL(probe_soa_k<8>, dim3(g), dim3(256), 0, 0, in, r8, ntiles, ctile);
      } else if (pl <= 5u) {
        hipLaunchKernelGGL(probe_k<5>, dim3(g), dim3(256), 0, 0, in, rec, ntiles, ctile);
      } else {
        hipLaunchKernelGGL(probe_k<8>, dim3(g), dim3(256), 0, 0, in, rec, ntiles, ctile);
      }
    };
    // untimed launches for warm_ms (the clocks settle, as bench.py does for the decode)
    float spent = 0.0f;
    while (spent < warm_ms) {
      if ((e = hipEventRecord(a, 0)) != hipSuccess) goto done;
      for (int r = 0; r < 10; r++) launch();
      if ((e = hipEventRecord(b, 0)) != hipSuccess || (e = hipEventSynchronize(b)) != hipSuccess) goto done;
      float ms = 0.0f;
      if ((e = hipEventElapsedTime(&ms, a, b)) != hipSuccess) goto done;
      spent += ms;
      if (ms <= 0.0f) break;
    }
    if ((e = hipEventRecord(a, 0)) != hipSuccess) goto done;
    for (int r = 0; r < reps; r++) launch();
    if ((e = hipEventRecord(b, 0)) != hipSuccess || (e = hipEventSynchronize(b)) != hipSuccess) goto done;
    float ms = 0.0f;
    if ((e = hipEventElapsedTime(&ms, a, b)) != hipSuccess) goto done;
    ms /= (float)reps;
    if ((e = hipGetLastError()) != hipSuccess) goto done;
    if (best == 0.0f || ms < best) best = ms;
  }
  *best_ms = best;
done:
  if (a) (void)hipEventDestroy(a);
  if (b) (void)hipEventDestroy(b);
  if (in) (void)hipFree(in);
  if (rec) (void)hipFree(rec);
  return (int)e;
}

// Diagnostics of the streaming structure (tools/): the same probe at a given
// number of workgroups per CU (wpc), with lds_per_wg bytes of dynamic LDS per workgroup (to cap
// the resident waves as a decode kernel's LDS does) and optionally every round copied to LDS
// before it is folded (commit).  *ms: mean launch time after warm_ms of untimed launches.
int gpd_probe_stream_ex(int device, uint32_t ntiles, uint32_t read_bytes_per_tile, int reps, float warm_ms,
                        uint32_t wpc, uint32_t lds_per_wg, int commit, float *ms_out) {
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return (int)e;
  const uint32_t ctile = (read_bytes_per_tile + 15u) / 16u;
  if (ctile == 0 || ctile > kMaxTileBytes / 16u || ntiles == 0 || reps <= 0 || wpc == 0) return (int)hipErrorInvalidValue;
  hipDeviceProp_t prop;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return (int)e;
  const uint32_t need = commit ? 4u * 8u * 64u * 16u : 0u;  // 4 waves x 8 chunks x 64 lanes
  const uint32_t lds = lds_per_wg > need ? lds_per_wg : need;
  v4u *in = nullptr, *rec = nullptr;
  hipEvent_t a = nullptr, b = nullptr;
  float ms = 0.0f, spent = 0.0f;
  const uint32_t g = (uint32_t)prop.multiProcessorCount * wpc;
  auto launch = [&] {
    if (commit) hipLaunchKernelGGL((probe_k<8, true>), dim3(g), dim3(256), lds, 0, in, rec, ntiles, ctile);
    else hipLaunchKernelGGL((probe_k<8, false>), dim3(g), dim3(256), lds, 0, in, rec, ntiles, ctile);
  };
  if ((e = hipMalloc(&in, (size_t)ntiles * ctile * 16u)) != hipSuccess) goto done;
  if ((e = hipMalloc(&rec, (size_t)ntiles * 2048u)) != hipSuccess) goto done;
  if ((e = hipMemset(in, 0x5a, (size_t)ntiles * ctile * 16u)) != hipSuccess) goto done;
  if ((e = hipEventCreate(&a)) != hipSuccess || (e = hipEventCreate(&b)) != hipSuccess) goto done;
  while (spent < warm_ms) {
    if ((e = hipEventRecord(a, 0)) != hipSuccess) goto done;
    for (int r = 0; r < 10; r++) launch();
    if ((e = hipEventRecord(b, 0)) != hipSuccess || (e = hipEventSynchronize(b)) != hipSuccess) goto done;
    if ((e = hipEventElapsedTime(&ms, a, b)) != hipSuccess) goto done;
    spent += ms;
    if (ms <= 0.0f) break;
  }
  if ((e = hipEventRecord(a, 0)) != hipSuccess) goto done;
  for (int r = 0; r < reps; r++) launch();
  if ((e = hipEventRecord(b, 0)) != hipSuccess || (e = hipEventSynchronize(b)) != hipSuccess) goto done;
  if ((e = hipEventElapsedTime(&ms, a, b)) != hipSuccess) goto done;
  if ((e = hipGetLastError()) != hipSuccess) goto done;
  *ms_out = ms / (float)reps;
done:
  if (a) (void)hipEventDestroy(a);
  if (b) (void)hipEventDestroy(b);
  if (in) (void)hipFree(in);
  if (rec) (void)hipFree(rec);
  return (int)e;
}

}  // extern "C"
