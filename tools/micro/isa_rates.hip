// Issue-rate microbenchmark for the integer VALU instructions the decode kernel leans on.
// Each lane runs 8 independent chains of one instruction; the throughput is reported as
// wave-instructions per SIMD per cycle relative to v_add_u32.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHAINS(OP)                                                                  \
  asm volatile(OP OP OP OP OP OP OP OP                                                \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(k) :);

template <int K>
__global__ void bench(uint32_t *out, int iters, uint32_t k) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; i++) {
    if constexpr (K == 0) {
      asm volatile(
          "v_add_u32 %0, %0, %8\n v_add_u32 %1, %1, %8\n v_add_u32 %2, %2, %8\n v_add_u32 %3, %3, %8\n"
          "v_add_u32 %4, %4, %8\n v_add_u32 %5, %5, %8\n v_add_u32 %6, %6, %8\n v_add_u32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 1) {
      asm volatile(
          "v_mul_lo_u32 %0, %0, %8\n v_mul_lo_u32 %1, %1, %8\n v_mul_lo_u32 %2, %2, %8\n v_mul_lo_u32 %3, %3, %8\n"
          "v_mul_lo_u32 %4, %4, %8\n v_mul_lo_u32 %5, %5, %8\n v_mul_lo_u32 %6, %6, %8\n v_mul_lo_u32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 2) {
      asm volatile(
          "v_mul_hi_u32 %0, %0, %8\n v_mul_hi_u32 %1, %1, %8\n v_mul_hi_u32 %2, %2, %8\n v_mul_hi_u32 %3, %3, %8\n"
          "v_mul_hi_u32 %4, %4, %8\n v_mul_hi_u32 %5, %5, %8\n v_mul_hi_u32 %6, %6, %8\n v_mul_hi_u32 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 3) {
      asm volatile(
          "v_mul_u32_u24 %0, %0, %8\n v_mul_u32_u24 %1, %1, %8\n v_mul_u32_u24 %2, %2, %8\n v_mul_u32_u24 %3, %3, %8\n"
          "v_mul_u32_u24 %4, %4, %8\n v_mul_u32_u24 %5, %5, %8\n v_mul_u32_u24 %6, %6, %8\n v_mul_u32_u24 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 4) {
      asm volatile(
          "v_dot4_u32_u8 %0, %0, %8, %0\n v_dot4_u32_u8 %1, %1, %8, %1\n v_dot4_u32_u8 %2, %2, %8, %2\n v_dot4_u32_u8 %3, %3, %8, %3\n"
          "v_dot4_u32_u8 %4, %4, %8, %4\n v_dot4_u32_u8 %5, %5, %8, %5\n v_dot4_u32_u8 %6, %6, %8, %6\n v_dot4_u32_u8 %7, %7, %8, %7\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 5) {
      asm volatile(
          "v_dot2_u32_u16 %0, %0, %8, %0\n v_dot2_u32_u16 %1, %1, %8, %1\n v_dot2_u32_u16 %2, %2, %8, %2\n v_dot2_u32_u16 %3, %3, %8, %3\n"
          "v_dot2_u32_u16 %4, %4, %8, %4\n v_dot2_u32_u16 %5, %5, %8, %5\n v_dot2_u32_u16 %6, %6, %8, %6\n v_dot2_u32_u16 %7, %7, %8, %7\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 6) {
      asm volatile(
          "v_perm_b32 %0, %0, %8, %8\n v_perm_b32 %1, %1, %8, %8\n v_perm_b32 %2, %2, %8, %8\n v_perm_b32 %3, %3, %8, %8\n"
          "v_perm_b32 %4, %4, %8, %8\n v_perm_b32 %5, %5, %8, %8\n v_perm_b32 %6, %6, %8, %8\n v_perm_b32 %7, %7, %8, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 7) {
      asm volatile(
          "v_mul_hi_u32_u24 %0, %0, %8\n v_mul_hi_u32_u24 %1, %1, %8\n v_mul_hi_u32_u24 %2, %2, %8\n v_mul_hi_u32_u24 %3, %3, %8\n"
          "v_mul_hi_u32_u24 %4, %4, %8\n v_mul_hi_u32_u24 %5, %5, %8\n v_mul_hi_u32_u24 %6, %6, %8\n v_mul_hi_u32_u24 %7, %7, %8\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    } else if constexpr (K == 8) {
      asm volatile(
          "v_bfe_u32 %0, %0, 3, 9\n v_bfe_u32 %1, %1, 3, 9\n v_bfe_u32 %2, %2, 3, 9\n v_bfe_u32 %3, %3, 3, 9\n"
          "v_bfe_u32 %4, %4, 3, 9\n v_bfe_u32 %5, %5, 3, 9\n v_bfe_u32 %6, %6, 3, 9\n v_bfe_u32 %7, %7, 3, 9\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(k));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 64-bit chains (v_mad_u64_u32, v_lshlrev_b64, v_lshl_add_u64)
template <int K>
__global__ void bench64(uint64_t *out, int iters, uint32_t k) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  for (int i = 0; i < iters; i++) {
    if constexpr (K == 0) {
      asm volatile(
          "v_mad_u64_u32 %0, s[0:1], %4, %4, %0\n v_mad_u64_u32 %1, s[0:1], %4, %4, %1\n"
          "v_mad_u64_u32 %2, s[0:1], %4, %4, %2\n v_mad_u64_u32 %3, s[0:1], %4, %4, %3\n"
          "v_mad_u64_u32 %0, s[0:1], %4, %4, %0\n v_mad_u64_u32 %1, s[0:1], %4, %4, %1\n"
          "v_mad_u64_u32 %2, s[0:1], %4, %4, %2\n v_mad_u64_u32 %3, s[0:1], %4, %4, %3\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(k) : "s0", "s1");
    } else if constexpr (K == 1) {
      asm volatile(
          "v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n v_lshlrev_b64 %3, 3, %3\n"
          "v_lshlrev_b64 %0, 3, %0\n v_lshlrev_b64 %1, 3, %1\n v_lshlrev_b64 %2, 3, %2\n v_lshlrev_b64 %3, 3, %3\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(k));
    } else if constexpr (K == 2) {
      asm volatile(
          "v_lshl_add_u64 %0, %0, 3, %0\n v_lshl_add_u64 %1, %1, 3, %1\n v_lshl_add_u64 %2, %2, 3, %2\n v_lshl_add_u64 %3, %3, 3, %3\n"
          "v_lshl_add_u64 %0, %0, 3, %0\n v_lshl_add_u64 %1, %1, 3, %1\n v_lshl_add_u64 %2, %2, 3, %2\n v_lshl_add_u64 %3, %3, 3, %3\n"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(k));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3;
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 4, threads = 256, iters = 4096;  // 4 waves/SIMD
  uint32_t *o32;
  uint64_t *o64;
  hipMalloc(&o32, blocks * threads * 4);
  hipMalloc(&o64, blocks * threads * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char *names[] = {"v_add_u32", "v_mul_lo_u32", "v_mul_hi_u32", "v_mul_u32_u24", "v_dot4_u32_u8",
                         "v_dot2_u32_u16", "v_perm_b32", "v_mul_hi_u32_u24", "v_bfe_u32"};
  void (*ks[])(uint32_t *, int, uint32_t) = {bench<0>, bench<1>, bench<2>, bench<3>, bench<4>,
                                             bench<5>, bench<6>, bench<7>, bench<8>};
  const double instrs = (double)blocks * (threads / 64) * iters * 8;  // wave-instructions
  const double simds = cus * 4.0;
  double base = 0;
  for (int k = 0; k < 9; k++) {
    hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(threads), 0, 0, o32, iters, 0x01010101u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[k], dim3(blocks), dim3(threads), 0, 0, o32, iters, 0x01010101u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double per_simd_ns = ms * 1e6 / (instrs / simds);
    if (k == 0) base = per_simd_ns;
    printf("%-18s %.3f ns/wave-instr/SIMD  cost %.2fx v_add\n", names[k], per_simd_ns, per_simd_ns / base);
  }
  const char *n64[] = {"v_mad_u64_u32", "v_lshlrev_b64", "v_lshl_add_u64"};
  void (*k64[])(uint64_t *, int, uint32_t) = {bench64<0>, bench64<1>, bench64<2>};
  for (int k = 0; k < 3; k++) {
    hipLaunchKernelGGL(k64[k], dim3(blocks), dim3(threads), 0, 0, o64, iters, 3u);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k64[k], dim3(blocks), dim3(threads), 0, 0, o64, iters, 3u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double per_simd_ns = ms * 1e6 / (instrs / simds);
    printf("%-18s %.3f ns/wave-instr/SIMD  cost %.2fx v_add\n", n64[k], per_simd_ns, per_simd_ns / base);
  }
  return 0;
}
