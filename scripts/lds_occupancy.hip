// Workgroups resident per CU as a function of dynamic LDS bytes (gfx950), measured: a grid of
// one-wave workgroups, each spinning ~30 us; the workgroups that start in the first round
// (start time within 15 us of the earliest) are the resident capacity of the 256 CUs.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/lds_occupancy scripts/lds_occupancy.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(64) void spin(unsigned long long* start, int vgpr_pad) {
  extern __shared__ float S[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) start[blockIdx.x] = t0;
  S[threadIdx.x] = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < 3000) {  // 100 MHz: 30 us
  }
  if (S[threadIdx.x] < -1.f) start[blockIdx.x] = 0;  // keep S live
}

int main() {
  const int nblk = 256 * 20;
  unsigned long long* d;
  hipMalloc(&d, sizeof(unsigned long long) * nblk);
  hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  std::vector<unsigned long long> h(nblk);
  for (int bytes : {12800, 12864, 12928, 12992, 13056, 13120, 13184, 13248, 13568, 13824, 14080, 14144, 14208, 14272, 14336, 10240, 10752, 11264}) {
    hipLaunchKernelGGL(spin, dim3(nblk), dim3(64), bytes, 0, d, 0);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    hipMemcpy(h.data(), d, sizeof(unsigned long long) * nblk, hipMemcpyDeviceToHost);
    const unsigned long long t0 = *std::min_element(h.begin(), h.end());
    int first = 0;
    for (auto t : h) first += (t - t0) < 1500;  // 15 us (the second round starts at 30 us)
    printf("LDS %6d B: first-round workgroups %5d = %.2f per CU (160 KiB / bytes = %.2f)\n", bytes, first,
           first / 256.0, 163840.0 / bytes);
  }
  return 0;
}
