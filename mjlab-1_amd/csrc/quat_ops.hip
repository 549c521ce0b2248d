// Batched quaternion product for the torch-side managers (tracking / jump terms).
//
// The reference's `quat_mul` (src/mjlab/utils/lab_api/math.py:526-563) is ~30 elementwise
// torch kernels over strided views; here one thread computes one product.  It uses the
// reference's 8-multiply operation order (ww, yy, zz, xx, qq) with FP contraction off, so
// every intermediate is rounded exactly as the separate torch kernels of the reference
// expression round it: bit-identical to that expression (restated in
// mjlab_amd/math_utils.py and tests/test_gpu_quat.py).
#include <hip/hip_runtime.h>

#include "../../include/mjx355_task.h"

namespace {

__global__ void k_quat_mul(const float4* __restrict__ a, const float4* __restrict__ b,
                           float4* __restrict__ out, long n) {
#pragma clang fp contract(off)
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float4 p = a[i], q = b[i];  // (w, x, y, z) in (x, y, z, w) slots
  const float w1 = p.x, x1 = p.y, y1 = p.z, z1 = p.w;
  const float w2 = q.x, x2 = q.y, y2 = q.z, z2 = q.w;
  const float ww = (z1 + x1) * (x2 + y2);
  const float yy = (w1 - y1) * (w2 + z2);
  const float zz = (w1 + y1) * (w2 - z2);
  const float xx = ww + yy + zz;
  const float qq = 0.5f * (xx + (z1 - x1) * (x2 - y2));
  float4 r;
  r.x = qq - ww + (z1 - y1) * (y2 - z2);
  r.y = qq - xx + (x1 + w1) * (x2 + w2);
  r.z = qq - yy + (w1 - x1) * (y2 + z2);
  r.w = qq - zz + (z1 + y1) * (w2 - x2);
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
