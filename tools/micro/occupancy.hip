// Residency probe (diagnostic, not product; round 6): how many 256-thread workgroups does the
// dispatcher keep on one CU at once for a given dynamic-LDS reservation and grid size?  Each
// workgroup counts itself in on its CU (HW_ID cu/sh/se + XCC_ID), records the running maximum,
// sleeps ~20 us so that co-resident workgroups overlap, and counts itself out.  Counters are
// plain vector atomics on global memory.
//   hipcc --offload-arch=gfx950 -O3 -o occupancy occupancy.hip
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

extern __shared__ uint32_t lds[];

constexpr int kKeys = 8 * 1024;

__global__ __launch_bounds__(256) void occ_k(uint32_t *cur, uint32_t *mx, uint32_t *seen, int sleeps) {
  // HW_ID (gfx9 layout): cu_id [11:8], sh_id [12], se_id [15:13]; XCC_ID [3:0]
  const uint32_t hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
  const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11));
  const uint32_t key = ((xcc & 15u) << 9) | (((hw >> 13) & 7u) << 5) | (((hw >> 12) & 1u) << 4) | ((hw >> 8) & 15u);
  if (threadIdx.x == 0) {
    const uint32_t v = atomicAdd(cur + key, 1u) + 1u;
    atomicMax(mx + key, v);
    atomicAdd(seen + key, 1u);
  }
  lds[threadIdx.x] = threadIdx.x;
  for (int s = 0; s < sleeps; s++) __builtin_amdgcn_s_sleep(127);
  __syncthreads();
  if (threadIdx.x == 0) atomicSub(cur + key, 1u);
}

int main() {
  uint32_t *cur, *mx, *seen;
  CK(hipMalloc(&cur, kKeys * 4));
  CK(hipMalloc(&mx, kKeys * 4));
  CK(hipMalloc(&seen, kKeys * 4));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("occupancy: %s %d CUs, sharedMemPerBlock %zu, maxSharedMemoryPerMultiProcessor %zu\n", prop.gcnArchName,
         cus, prop.sharedMemPerBlock, prop.maxSharedMemoryPerMultiProcessor);
  struct Case { uint32_t lds; int wpc; };
  const Case cases[] = {{1024, 2}, {1024, 4}, {20480, 2}, {20480, 4}, {20480, 16},
                        {40960, 4}, {40960, 16}, {54608, 3}, {54608, 12}, {53248, 12}, {52224, 12},
                        {81920, 2}, {81920, 8}, {80896, 8}, {163840, 2}};
  for (const Case &c : cases) {
    CK(hipMemset(cur, 0, kKeys * 4));
    CK(hipMemset(mx, 0, kKeys * 4));
    CK(hipMemset(seen, 0, kKeys * 4));
    hipLaunchKernelGGL(occ_k, dim3(cus * c.wpc), dim3(256), c.lds, 0, cur, mx, seen, 200);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> m(kKeys), s(kKeys);
    CK(hipMemcpy(m.data(), mx, kKeys * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s.data(), seen, kKeys * 4, hipMemcpyDeviceToHost));
    int used = 0, hist[40] = {0}, shist[40] = {0};
    for (int k = 0; k < kKeys; k++)
      if (s[k]) {
        used++;
        hist[m[k] < 39 ? m[k] : 39]++;
        shist[s[k] < 39 ? s[k] : 39]++;
      }
    printf("RESULT lds=%6u grid=%5d cus_used=%d max_resident_hist:", c.lds, cus * c.wpc, used);
    for (int i = 0; i < 40; i++)
      if (hist[i]) printf(" %d:%d", i, hist[i]);
    printf(" | wgs_per_cu_hist:");
    for (int i = 0; i < 40; i++)
      if (shist[i]) printf(" %d:%d", i, shist[i]);
    printf("\n");
    fflush(stdout);
  }
  return 0;
}
