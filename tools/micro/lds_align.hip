// LDS probe (diagnostic): cost of ds_read_b128 / b64 / b32 at 16-B-aligned vs misaligned
// byte addresses (gfx950 DS takes unaligned addresses; how fast?).
//   hipcc --offload-arch=gfx950 -O3 -o lds_align lds_align.hip && ./lds_align
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

struct __attribute__((packed, aligned(1))) U128 { uint32_t x, y, z, w; };
struct __attribute__((packed, aligned(1))) U64 { uint32_t x, y; };

template <int KIND>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters, uint32_t mis, uint32_t stride) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
  for (uint32_t i = threadIdx.x; i < 65536 / 4; i += 256) reinterpret_cast<uint32_t *>(lds)[i] = i * 2654435761u;
  __syncthreads();
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t a = wave * 16384 + lane * stride + mis, acc = 0;
  for (int it = 0; it < iters; it++) {
    const uint32_t ad = (a + (uint32_t)it * 16u) & 0xBFFFu;  // stay inside the wave's 16 KiB
    if (KIND == 0) {
      const U128 q = *reinterpret_cast<const U128 *>(lds + wave * 16384 + (ad & 0x3FFF));
      acc += q.x ^ q.y ^ q.z ^ q.w;
    } else if (KIND == 1) {
      const U64 q = *reinterpret_cast<const U64 *>(lds + wave * 16384 + (ad & 0x3FFF));
      acc += q.x ^ q.y;
    } else {
      acc += *reinterpret_cast<const uint32_t *>(lds + wave * 16384 + (ad & 0x3FFC) + (mis & 3));
    }
  }
  if (acc == 0x1234567u) out[threadIdx.x] = acc;
}

int main() {
  uint32_t *o;
  (void)hipMalloc(&o, 4096);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int iters = 4096, blocks = 256 * 4;
  const char *names[] = {"b128", "b64", "b32"};
  for (int kind = 0; kind < 3; kind++)
    for (uint32_t stride : {16u, 64u, 80u})
      for (uint32_t mis : {0u, 2u, 4u, 8u, 14u}) {
        auto f = [&] {
          if (kind == 0) hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, o, iters, mis, stride);
          if (kind == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, o, iters, mis, stride);
          if (kind == 2) hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, o, iters, mis, stride);
        };
        f();
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        f();
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        const double per = ms * 1e6 / ((double)blocks * 4 * iters / (256.0 * 4));  // ns per wave-read per CU-SIMD set
        printf("%s stride %3u mis %2u: %.3f ms  %.2f ns/wave-read/CU\n", names[kind], stride, mis, ms,
               ms * 1e6 / ((double)blocks * 4 * iters / 256.0));
        (void)per;
      }
  return 0;
}
