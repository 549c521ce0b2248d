"""`mjx_quat_mul` (csrc/quat_ops.hip) against the torch expression of the reference's
quat_mul (src/mjlab/utils/lab_api/math.py:526-563, the 8-multiply form, restated below in
eager torch): bit-identical, with broadcasting, misaligned views and the empty batch."""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _torch_quat_mul(q1, q2):
  q1, q2 = torch.broadcast_tensors(q1, q2)
  w1, x1, y1, z1 = q1.unbind(-1)
  w2, x2, y2, z2 = q2.unbind(-1)
  ww = (z1 + x1) * (x2 + y2)
  yy = (w1 - y1) * (w2 + z2)
  zz = (w1 + y1) * (w2 - z2)
  xx = ww + yy + zz
  qq = 0.5 * (xx + (z1 - x1) * (x2 - y2))
  return torch.stack([qq - ww + (z1 - y1) * (y2 - z2), qq - xx + (x1 + w1) * (x2 + w2),
                      qq - yy + (w1 - x1) * (y2 + z2), qq - zz + (z1 + y1) * (w2 - x2)], dim=-1)


def _hamilton(q1, q2):
  w1, x1, y1, z1 = q1.unbind(-1)
  w2, x2, y2, z2 = q2.unbind(-1)
  return torch.stack([
    w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
    w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
    w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
    w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], dim=-1)


def test_quat_mul_bit_identical(gpu_device):
  from mjlab_amd.math_utils import quat_mul
  g = torch.Generator(device=gpu_device).manual_seed(0)
  a = torch.randn(4096, 37, 4, device=gpu_device, generator=g)
  b = torch.randn(4096, 37, 4, device=gpu_device, generator=g)
  assert torch.equal(quat_mul(a, b), _torch_quat_mul(a, b))
  # broadcasting: one quaternion per env against per-body quaternions
  c = a[:, :1, :]
  assert torch.equal(quat_mul(c, b), _torch_quat_mul(c, b))
  assert torch.equal(quat_mul(b, c.expand(-1, 37, -1)), _torch_quat_mul(b, c))
  # and it is the Hamilton product (to rounding)
  torch.testing.assert_close(quat_mul(a, b), _hamilton(a, b), rtol=1e-4, atol=1e-4)


def test_quat_mul_misaligned_and_empty(gpu_device):
  from mjlab_amd.math_utils import quat_mul
  root = torch.randn(64, 13, device=gpu_device)
  q = root[:, 3:7]  # row view starting mid-float4
  r = torch.randn(64, 4, device=gpu_device)
  assert torch.equal(quat_mul(q, r), _torch_quat_mul(q, r))
  flat = torch.randn(4 * 9 + 1, device=gpu_device)[1:].view(9, 4)  # contiguous, misaligned
  assert torch.equal(quat_mul(flat, flat), _torch_quat_mul(flat, flat))
  e = torch.empty(0, 4, device=gpu_device)
  assert quat_mul(e, e).shape == (0, 4)
