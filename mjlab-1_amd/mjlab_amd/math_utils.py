"""Batched quaternion / sampling helpers (wxyz convention) used by entity views and terms.

Same conventions and semantics as the torch helpers the reference takes from Isaac Lab
(`src/mjlab/utils/lab_api/math.py:102,166,275,318,527,629,651,1360`).
"""

from __future__ import annotations

import torch


_quat_mul_fn = None


def _quat_mul_hip(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  """One `mjx_quat_mul` launch (csrc/quat_ops.hip) instead of ~30 strided torch kernels;
  bit-identical to the reference expression below.  Raises if the HIP library is missing."""
  global _quat_mul_fn
  if _quat_mul_fn is None:
    import ctypes
    from ._lib import lib
    f = lib().mjx_quat_mul
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p]
    f.restype = ctypes.c_int
    _quat_mul_fn = f
  a, b = torch.broadcast_tensors(q1, q2)
  # the kernel reads float4 rows: contiguous and 16-byte aligned (a view may start mid-row)
  a = a.contiguous() if a.data_ptr() % 16 == 0 else a.clone(memory_format=torch.contiguous_format)
  b = b.contiguous() if b.data_ptr() % 16 == 0 else b.clone(memory_format=torch.contiguous_format)
  out = torch.empty(a.shape, dtype=torch.float32, device=a.device)
  rc = _quat_mul_fn(a.data_ptr(), b.data_ptr(), out.data_ptr(), out.numel() // 4,
                    torch.cuda.current_stream(a.device).cuda_stream)
  if rc != 0:
    raise RuntimeError(f"mjx_quat_mul failed ({rc})")
  return out


def quat_mul(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  """`utils/lab_api/math.py:526-563`: the 8-multiply (ww, yy, zz, xx, qq) product, same
  operation order.  Unlike the reference, inputs broadcast against each other (the
  reference raises ValueError on any shape mismatch); non-broadcastable shapes and a last
  dim other than 4 raise ValueError."""
  try:
    shape = torch.broadcast_shapes(q1.shape, q2.shape)
  except RuntimeError as e:
    raise ValueError(f"Expected input quaternion shape mismatch: {q1.shape} != {q2.shape}.") from e
  if len(shape) == 0 or shape[-1] != 4:
    raise ValueError(f"quat_mul: last dim must be 4, got {tuple(shape)}")
  if (q1.is_cuda and q1.dtype == torch.float32 and q2.dtype == torch.float32
      and q1.device == q2.device):
    return _quat_mul_hip(q1, q2)
  w1, x1, y1, z1 = q1.unbind(-1)
  w2, x2, y2, z2 = q2.unbind(-1)
  ww = (z1 + x1) * (x2 + y2)
  yy = (w1 - y1) * (w2 + z2)
  zz = (w1 + y1) * (w2 - z2)
  xx = ww + yy + zz
  qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
  w = qq - ww + (z1 - y1) * (y2 - z2)
  x = qq - xx + (x1 + w1) * (x2 + w2)
  y = qq - yy + (w1 - x1) * (y2 + z2)
  z = qq - zz + (z1 + y1) * (w2 - x2)
  return torch.stack([w, x, y, z], dim=-1)


def quat_apply(quat: torch.Tensor, vec: torch.Tensor) -> torch.Tensor:
  """Rotate `vec` by `quat` (v' = q v q*)."""
  vec = vec.expand(quat.shape[:-1] + (3,)) if vec.dim() < quat.dim() else vec
  w = quat[..., :1]
  xyz = quat[..., 1:]
  t = 2.0 * torch.cross(xyz, vec, dim=-1)
  return vec + w * t + torch.cross(xyz, t, dim=-1)


def quat_apply_inverse(quat: torch.Tensor, vec: torch.Tensor) -> torch.Tensor:
  """Rotate `vec` by the inverse of `quat`."""
  vec = vec.expand(quat.shape[:-1] + (3,)) if vec.dim() < quat.dim() else vec
  w = quat[..., :1]
  xyz = quat[..., 1:]
  t = 2.0 * torch.cross(xyz, vec, dim=-1)
  return vec - w * t + torch.cross(xyz, t, dim=-1)


def quat_from_euler_xyz(roll: torch.Tensor, pitch: torch.Tensor, yaw: torch.Tensor):
  cr, sr = torch.cos(roll * 0.5), torch.sin(roll * 0.5)
  cp, sp = torch.cos(pitch * 0.5), torch.sin(pitch * 0.5)
  cy, sy = torch.cos(yaw * 0.5), torch.sin(yaw * 0.5)
  return torch.stack([cy * cr * cp + sy * sr * sp,
                      cy * sr * cp - sy * cr * sp,
                      cy * cr * sp + sy * sr * cp,
                      sy * cr * cp - cy * sr * sp], dim=-1)


def quat_from_matrix(m: torch.Tensor) -> torch.Tensor:
  """Rotation matrix (..., 9) or (..., 3, 3) -> quaternion (w, x, y, z), as
  `utils/lab_api/math.py:318-372`: of the four quaternion components the largest in magnitude
  is formed from the trace-like sum, the others from the matrix's off-diagonal sums and
  differences divided by it (the best-conditioned candidate; that component comes out
  positive)."""
  if m.shape[-1] == 9:
    m = m.reshape(m.shape[:-1] + (3, 3))
  m00, m01, m02 = m[..., 0, 0], m[..., 0, 1], m[..., 0, 2]
  m10, m11, m12 = m[..., 1, 0], m[..., 1, 1], m[..., 1, 2]
  m20, m21, m22 = m[..., 2, 0], m[..., 2, 1], m[..., 2, 2]
  four = torch.stack([1 + m00 + m11 + m22, 1 + m00 - m11 - m22, 1 - m00 + m11 - m22,
                      1 - m00 - m11 + m22], dim=-1)
  mag = torch.sqrt(torch.clamp(four, min=0))  # 2 |q_i|
  rows = torch.stack([
    torch.stack([four[..., 0], m21 - m12, m02 - m20, m10 - m01], dim=-1),
    torch.stack([m21 - m12, four[..., 1], m10 + m01, m02 + m20], dim=-1),
    torch.stack([m02 - m20, m10 + m01, four[..., 2], m12 + m21], dim=-1),
    torch.stack([m10 - m01, m20 + m02, m21 + m12, four[..., 3]], dim=-1)], dim=-2)
  k = mag.argmax(dim=-1, keepdim=True)
  best = torch.gather(rows, -2, k.unsqueeze(-1).expand(*k.shape[:-1], 1, 4)).squeeze(-2)
  return best / (2.0 * torch.gather(mag, -1, k).clamp(min=0.1))


def matrix_from_quat(q: torch.Tensor) -> torch.Tensor:
  w, x, y, z = q.unbind(-1)
  return torch.stack([
    1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
    2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
    2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=-1
  ).reshape(q.shape[:-1] + (3, 3))


def wrap_to_pi(angles: torch.Tensor) -> torch.Tensor:
  wrapped = torch.remainder(angles, 2 * torch.pi)
  return torch.where(wrapped > torch.pi, wrapped - 2 * torch.pi, wrapped)


def sample_uniform(lower, upper, size, device, generator=None) -> torch.Tensor:
  if isinstance(size, int):
    size = (size,)
  return torch.rand(*size, device=device, generator=generator) * (upper - lower) + lower


def yaw_quat(quat: torch.Tensor) -> torch.Tensor:
  w, x, y, z = quat.unbind(-1)
  yaw = torch.atan2(2 * (w * z + x * y), 1 - 2 * (y * y + z * z))
  out = torch.zeros_like(quat)
  out[..., 0] = torch.cos(yaw / 2)
  out[..., 3] = torch.sin(yaw / 2)
  return out


def quat_conjugate(q: torch.Tensor) -> torch.Tensor:
  return torch.cat((q[..., 0:1], -q[..., 1:]), dim=-1)


def quat_inv(q: torch.Tensor, eps: float = 1e-9) -> torch.Tensor:
  """`math.py:261-271`: conjugate / |q|^2."""
  return quat_conjugate(q) / q.pow(2).sum(dim=-1, keepdim=True).clamp(min=eps)


def quat_unique(q: torch.Tensor) -> torch.Tensor:
  return torch.where(q[..., 0:1] < 0, -q, q)


def axis_angle_from_quat(quat: torch.Tensor, eps: float = 1.0e-6) -> torch.Tensor:
  """`math.py:478-506`: log map, shortest arc (w >= 0), Taylor branch near zero."""
  quat = quat * (1.0 - 2.0 * (quat[..., 0:1] < 0.0))
  mag = torch.linalg.norm(quat[..., 1:], dim=-1)
  half = torch.atan2(mag, quat[..., 0])
  angle = 2.0 * half
  s = torch.where(angle.abs() > eps, torch.sin(half) / angle, 0.5 - angle * angle / 48)
  return quat[..., 1:4] / s.unsqueeze(-1)


def quat_box_minus(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  """`math.py:590-604`: log(q1 * conj(q2))."""
  return axis_angle_from_quat(quat_mul(q1, quat_conjugate(q2)))


def quat_error_magnitude(q1: torch.Tensor, q2: torch.Tensor) -> torch.Tensor:
  """`math.py:688-699`: |box_minus(q1, q2)| (rotation angle between the two)."""
  return torch.norm(quat_box_minus(q1, q2), dim=-1)


def subtract_frame_transforms(t01, q01, t02=None, q02=None):
  """`math.py:832-863`: T12 = T01^-1 * T02."""
  q10 = quat_inv(q01)
  q12 = quat_mul(q10, q02) if q02 is not None else q10
  t12 = quat_apply(q10, t02 - t01) if t02 is not None else quat_apply(q10, -t01)
  return t12, q12
