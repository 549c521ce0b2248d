// Batched quaternion product for the torch-side managers (tracking / jump terms).
//
// The reference's `quat_mul` (src/mjlab/utils/lab_api/math.py:275) is ~30 elementwise torch
// kernels over strided views; here one thread computes one product.  FP contraction is off
// so each term is rounded exactly as the separate torch mul/add/sub kernels round it: the
// result is bit-identical to the torch expression in mjlab_amd/math_utils.py.
#include <hip/hip_runtime.h>

#include "../../include/mjx355_task.h"

namespace {

__global__ void k_quat_mul(const float4* __restrict__ a, const float4* __restrict__ b,
                           float4* __restrict__ out, long n) {
#pragma clang fp contract(off)
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = a[i], q = b[i];  // (w, x, y, z) in (x, y, z, w) slots
  float4 r;
  r.x = p.x * q.x - p.y * q.y - p.z * q.z - p.w * q.w;
  r.y = p.x * q.y + p.y * q.x + p.z * q.w - p.w * q.z;
  r.z = p.x * q.z - p.y * q.w + p.z * q.x + p.w * q.y;
  r.w = p.x * q.w + p.y * q.z - p.z * q.y + p.w * q.x;
  out[i] = r;
}

}  // namespace

extern "C" int mjx_quat_mul(const float* q1, const float* q2, float* out, long n, void* stream) {
  if (n < 0 || (n > 0 && (!q1 || !q2 || !out))) return -1;
  if (((uintptr_t)q1 | (uintptr_t)q2 | (uintptr_t)out) & 15) return -2;  // float4 rows
  if (n == 0) return 0;
  hipLaunchKernelGGL(k_quat_mul, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, reinterpret_cast<const float4*>(q1),
                     reinterpret_cast<const float4*>(q2), reinterpret_cast<float4*>(out), n);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
