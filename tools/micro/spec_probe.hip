// Wave-specialisation probe (diagnostic, not product): does splitting a workgroup's 4 waves into
// 2 streaming waves (global loads -> LDS) and 2 decoding waves (LDS -> VALU -> result stores),
// double-buffered through LDS with one barrier per step, move config 2's traffic faster than
// every wave doing both (the rs_kernel shape)?  The 2-workgroup streaming probe is 8 % faster
// than the 4-workgroup one (fewer concurrent streams); specialisation keeps 2
// streams per SIMD while the decode's latency is hidden by other waves.
//   uniform : 4 waves per workgroup, each: tile -> registers -> LDS -> synthetic decode -> stores
//   special : waves 0,1 stream tiles into LDS for waves 2,3, which decode and store
// Traffic per tile as config 2: 64 packets x 72 B read (4,608 B), 64 x 32 B written.  The
// synthetic decode reads four 16-B words per lane from LDS at its packet's offset and runs
// `iters` rounds of four independent multiply-xor chains (~ the fast path's VALU per tile).
//   hipcc --offload-arch=gfx950 -O3 -o spec_probe spec_probe.hip && ./spec_probe
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

constexpr uint32_t kTileChunks = 288;  // 4,608 B / 16
constexpr uint32_t kNc = 5;            // 16-B chunks per lane per tile (5 x 64 >= 288)

__device__ __forceinline__ uint32_t decode(const uint8_t *lds, uint32_t lane, uint32_t iters) {
  const uint32_t a = (lane * 72u) & ~15u;  // the lane's packet, aligned reads
  const v4u q0 = *reinterpret_cast<const v4u *>(lds + a), q1 = *reinterpret_cast<const v4u *>(lds + a + 16);
  const v4u q2 = *reinterpret_cast<const v4u *>(lds + a + 32), q3 = *reinterpret_cast<const v4u *>(lds + a + 48);
  uint32_t x = q0.x ^ q1.y, y = q0.z ^ q2.x, z = q1.w ^ q3.y, w = q2.z ^ q3.w;
  for (uint32_t i = 0; i < iters; i++) {
    x = x * 0x1b3u ^ (y >> 3);
    y = y * 0x2c9u ^ (z >> 5);
    z = z * 0x3e7u ^ (w >> 7);
    w = w * 0x4f1u ^ (x >> 11);
  }
  return x ^ y ^ z ^ w;
}

__device__ __forceinline__ void store_res(v4u *out, uint64_t i, uint32_t h) {
  __builtin_nontemporal_store(v4u{h, h ^ 1u, h * 3u, 0u}, out + 2 * i);
  __builtin_nontemporal_store(v4u{h * 5u, 0u, h * 7u, 0u}, out + 2 * i + 1);
}

// DESC: the tile's bytes are 4 KiB of frames plus its 64 descriptors as two separate u32
// arrays (offset, caplen: the real batch layout), loaded two tiles ahead with 4-B loads and
// reduced over the wave (the window planning's wave max) — the rs_kernel skeleton's shape
// DESC 2: the same descriptors as ONE 16-B load per lane (lanes 0-15: the tile's 256 B of
// offsets, 16-31: its caplens; lanes 32-63 repeat them), spread to the packet lanes with
// ds_bpermute — one memory instruction per tile instead of two
template <int DESC>
__global__ __launch_bounds__(256) void uniform_k(const v4u *__restrict__ in, v4u *out, uint32_t ntiles,
                                                 uint32_t iters, const uint32_t *off, const uint32_t *len) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][kNc * 1024];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint32_t nw = gridDim.x * 4u;
  uint8_t *buf = lds[wave];
  constexpr uint32_t kChunks = DESC ? 256u : kTileChunks;
  constexpr uint32_t kN = DESC ? 4u : kNc;
  uint32_t t = blockIdx.x * 4u + wave;
  uint32_t oa = 0, ca = 0, ob = 0, cb = 0;
  v4u da{0u, 0u, 0u, 0u}, db{0u, 0u, 0u, 0u};
  auto dld = [&](uint32_t u) -> v4u {
    const uint32_t *src = (lane & 16u) ? len : off;
    return __builtin_nontemporal_load(reinterpret_cast<const v4u *>(src + (uint64_t)u * 64u) + (lane & 15u));
  };
  if (DESC == 1) {
    const uint32_t t1 = t + nw < ntiles ? t + nw : t;
    oa = __builtin_nontemporal_load(off + (uint64_t)t * 64u + lane);
    ca = __builtin_nontemporal_load(len + (uint64_t)t * 64u + lane);
    ob = __builtin_nontemporal_load(off + (uint64_t)t1 * 64u + lane);
    cb = __builtin_nontemporal_load(len + (uint64_t)t1 * 64u + lane);
  } else if (DESC == 2) {
    da = dld(t);
    db = dld(t + nw < ntiles ? t + nw : t);
  }
  for (; t < ntiles; t += nw) {
    uint32_t hi = 0;
    if (DESC == 2) {  // lane l's offset: component l & 3 of lane l >> 2; caplen: of lane 16 + (l >> 2)
      const int so = (int)((lane >> 2) << 2), sc = (int)((16u + (lane >> 2)) << 2);
      const uint32_t k = lane & 3u;
      uint32_t o4[4], c4[4];
      o4[0] = __builtin_amdgcn_ds_bpermute(so, (int)da.x); o4[1] = __builtin_amdgcn_ds_bpermute(so, (int)da.y);
      o4[2] = __builtin_amdgcn_ds_bpermute(so, (int)da.z); o4[3] = __builtin_amdgcn_ds_bpermute(so, (int)da.w);
      c4[0] = __builtin_amdgcn_ds_bpermute(sc, (int)da.x); c4[1] = __builtin_amdgcn_ds_bpermute(sc, (int)da.y);
      c4[2] = __builtin_amdgcn_ds_bpermute(sc, (int)da.z); c4[3] = __builtin_amdgcn_ds_bpermute(sc, (int)da.w);
      oa = k == 0 ? o4[0] : k == 1 ? o4[1] : k == 2 ? o4[2] : o4[3];
      ca = k == 0 ? c4[0] : k == 1 ? c4[1] : k == 2 ? c4[2] : c4[3];
      da = db;
      db = dld(t + 2u * nw < ntiles ? t + 2u * nw : t);
    }
    if (DESC) {  // this tile's extent from its descriptors (a wave max), then the next-next tile's
      uint32_t e = oa + ca;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) e = max(e, (uint32_t)__shfl_xor((int)e, o));
      hi = __builtin_amdgcn_readfirstlane(e) & 3u;
      if (DESC == 1) {
        oa = ob;
        ca = cb;
        const uint32_t t2 = t + 2u * nw < ntiles ? t + 2u * nw : t;
        ob = __builtin_nontemporal_load(off + (uint64_t)t2 * 64u + lane);
        cb = __builtin_nontemporal_load(len + (uint64_t)t2 * 64u + lane);
      }
    }
    v4u v[kN];
#pragma unroll
    for (uint32_t j = 0; j < kN; j++) {
      const uint32_t c = 64u * j + lane;
      v[j] = __builtin_nontemporal_load(in + (uint64_t)t * kChunks + (c < kChunks ? c : 0u) + hi);
    }
#pragma unroll
    for (uint32_t j = 0; j < kN; j++) *reinterpret_cast<v4u *>(buf + 1024u * j + 16u * lane) = v[j];
    store_res(out, (uint64_t)t * 64u + lane, decode(buf, lane, iters));
  }
}

// waves 0,1 stream for waves 2,3 (producer p serves consumer p + 2); every consumer takes
// `steps` tiles (the host makes ntiles = steps x consumers), one barrier per step
__global__ __launch_bounds__(256) void special_k(const v4u *__restrict__ in, v4u *out, uint32_t steps,
                                                 uint32_t iters) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2][2][kNc * 1024];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const bool prod = wave < 2u;
  const uint32_t pair = wave & 1u;
  const uint32_t cons = blockIdx.x * 2u + pair;  // the consumer id this wave belongs to
  const uint32_t ncons = gridDim.x * 2u;
  auto tile = [&](uint32_t s) { return s * ncons + cons; };
  v4u v[kNc];
  auto load = [&](uint32_t s) {
#pragma unroll
    for (uint32_t j = 0; j < kNc; j++) {
      const uint32_t c = 64u * j + lane;
      v[j] = __builtin_nontemporal_load(in + (uint64_t)tile(s) * kTileChunks + (c < kTileChunks ? c : 0u));
    }
  };
  if (prod) load(0);
  for (uint32_t s = 0; s < steps; s++) {
    if (prod) {
      uint8_t *buf = lds[pair][s & 1u];
#pragma unroll
      for (uint32_t j = 0; j < kNc; j++) *reinterpret_cast<v4u *>(buf + 1024u * j + 16u * lane) = v[j];
      if (s + 1u < steps) load(s + 1u);
    }
    __syncthreads();
    if (!prod) store_res(out, (uint64_t)tile(s) * 64u + lane, decode(lds[pair][s & 1u], lane, iters));
  }
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < 100; r++) f();  // clock settle
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < reps; r++) f();
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ms / reps;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 50;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const uint32_t ntiles = 1u << 18;  // 2^24 packets
  v4u *in = nullptr, *out = nullptr;
  CK(hipMalloc(&in, (size_t)ntiles * kTileChunks * 16u));
  CK(hipMemset(in, 0x5a, (size_t)ntiles * kTileChunks * 16u));
  CK(hipMalloc(&out, (size_t)ntiles * 64u * 32u));
  uint32_t *offs = nullptr, *lens = nullptr;  // DESC: 2^24 descriptors (offset = 64 i, caplen 64)
  CK(hipMalloc(&offs, (size_t)ntiles * 64u * 4u));
  CK(hipMalloc(&lens, (size_t)ntiles * 64u * 4u));
  CK(hipMemset(offs, 0, (size_t)ntiles * 64u * 4u));
  CK(hipMemset(lens, 0x40, (size_t)ntiles * 64u * 4u));
  const double bytes = (double)ntiles * 64.0 * 104.0;
  printf("spec_probe: %s %d CUs, %u tiles (config 2's traffic)\n", prop.gcnArchName, cus, ntiles);
  for (uint32_t iters : {0u, 32u}) {
    for (int wg : {2, 3, 4}) {
      const uint32_t blocks = (uint32_t)(cus * wg);
      const float tu = timeit([&] { hipLaunchKernelGGL(uniform_k<0>, dim3(blocks), dim3(256), 0, 0, in, out, ntiles, iters, offs, lens); }, reps);
      const float td = timeit([&] { hipLaunchKernelGGL(uniform_k<1>, dim3(blocks), dim3(256), 0, 0, in, out, ntiles, iters, offs, lens); }, reps);
      const float t2 = timeit([&] { hipLaunchKernelGGL(uniform_k<2>, dim3(blocks), dim3(256), 0, 0, in, out, ntiles, iters, offs, lens); }, reps);
      printf("RESULT iters=%2u wg_per_cu=%d desc16_ms=%.4f (%.3f TB/s)\n", iters, wg, t2, bytes / (t2 * 1e-3) / 1e12);
      // special: ntiles must split evenly over the consumers
      const uint32_t ncons = blocks * 2u;
      float ts = -1.f;
      if (ntiles % ncons == 0u) {
        const uint32_t steps = ntiles / ncons;
        ts = timeit([&] { hipLaunchKernelGGL(special_k, dim3(blocks), dim3(256), 0, 0, in, out, steps, iters); }, reps);
      }
      printf("RESULT iters=%2u wg_per_cu=%d uniform_ms=%.4f (%.3f TB/s) desc_ms=%.4f (%.3f TB/s) special_ms=%.4f (%.3f TB/s)\n",
             iters, wg, tu, bytes / (tu * 1e-3) / 1e12, td, bytes / (td * 1e-3) / 1e12, ts,
             ts > 0 ? bytes / (ts * 1e-3) / 1e12 : 0.0);
    }
  }
  CK(hipFree(in));
  CK(hipFree(out));
  CK(hipFree(offs));
  CK(hipFree(lens));
  return 0;
}
