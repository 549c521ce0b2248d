"""Host-side manager / MDP logic on CPU tensors, against numpy restatements of the
reference formulas (each test cites the reference file:line it restates).

Parity of these terms is pinned by formula restatement only: running the reference's
Python to produce golden vectors was refused in this environment.
"""

import math
from types import SimpleNamespace as ns

import numpy as np
import pytest
import torch

from mjlab_amd import mdp
from mjlab_amd.managers import resolve_matching_names, resolve_matching_names_values
from mjlab_amd.math_utils import (matrix_from_quat, quat_apply, quat_apply_inverse,
                                  quat_from_euler_xyz, quat_from_matrix, quat_mul, wrap_to_pi,
                                  yaw_quat)

N, J, B, S = 48, 29, 32, 2
rng = np.random.default_rng(0)


def _t(a):
  return torch.as_tensor(np.asarray(a, dtype=np.float32))


def _unit(*shape):
  q = rng.standard_normal((*shape, 4)).astype(np.float32)
  return q / np.linalg.norm(q, axis=-1, keepdims=True)


class _Sensor:
  def __init__(self, **data):
    self.data = ns(**data)
    self.first = None

  def compute_first_contact(self, dt, abs_tol=1e-8):
    return self.first


@pytest.fixture()
def env():
  g = rng.standard_normal((N, 3)).astype(np.float32)
  g /= np.linalg.norm(g, axis=-1, keepdims=True)
  cmd = rng.standard_normal((N, 3)).astype(np.float32)
  cmd[:5] = 0.0
  lo = -np.abs(rng.standard_normal((N, J))) - 0.2
  data = ns(root_link_lin_vel_b=_t(rng.standard_normal((N, 3))),
            root_link_ang_vel_b=_t(rng.standard_normal((N, 3))), projected_gravity_b=_t(g),
            body_link_quat_w=_t(_unit(N, B)), gravity_vec_w=_t([0, 0, -1]),
            body_link_ang_vel_w=_t(rng.standard_normal((N, B, 3))),
            site_pos_w=_t(np.abs(rng.standard_normal((N, S, 3))) * 0.2),
            site_lin_vel_w=_t(rng.standard_normal((N, S, 3))),
            joint_pos=_t(rng.standard_normal((N, J)) * 0.5), joint_vel=_t(rng.standard_normal((N, J))),
            default_joint_pos=_t(rng.standard_normal((N, J)) * 0.1),
            default_joint_vel=torch.zeros(N, J),
            soft_joint_pos_limits=_t(np.stack([lo, lo + 0.4 + np.abs(rng.standard_normal((N, J)))], -1)),
            root_link_pos_w=_t(np.abs(rng.standard_normal((N, 3))) * 0.8))
  feet = _Sensor(found=_t((rng.uniform(size=(N, S)) < 0.5) * rng.integers(1, 3, (N, S))),
                 current_air_time=_t(np.where(rng.uniform(size=(N, S)) < 0.5, 0, rng.uniform(0, 0.8, (N, S)))),
                 force=_t(rng.standard_normal((N, S, 3)) * 50))
  feet.first = torch.as_tensor(rng.uniform(size=(N, S)) < 0.3)
  scene = {"robot": ns(data=data), "feet": feet,
           "self_collision": _Sensor(found=_t(rng.integers(0, 3, (N, 1)))),
           "nonfoot": _Sensor(found=_t(rng.uniform(size=(N, 5)) < 0.1)),
           "angmom": ns(data=_t(rng.standard_normal((N, 3))))}
  c = _t(cmd)
  return ns(scene=scene, command_manager=ns(get_command=lambda name: c),
            action_manager=ns(action=_t(rng.standard_normal((N, J))),
                              prev_action=_t(rng.standard_normal((N, J)))),
            extras={"log": {}}, step_dt=0.02, num_envs=N, device="cpu",
            episode_length_buf=torch.as_tensor(rng.integers(990, 1010, N)), max_episode_length=1000)


def cfg(**kw):
  d = dict(name="robot", body_ids=slice(None), site_ids=slice(None), joint_ids=slice(None))
  d.update(kw)
  return ns(**d)


def _np(env, *path):
  x = env
  for p in path:
    x = x[p] if isinstance(x, dict) else getattr(x, p)
  return x.numpy().astype(np.float64)


def _active(c, thr):
  return ((np.linalg.norm(c[:, :2], axis=1) + np.abs(c[:, 2])) > thr).astype(np.float64)


def test_track_velocity_terms(env):
  """tasks/velocity/mdp/rewards.py:23-60."""
  c = env.command_manager.get_command("t").numpy().astype(np.float64)
  v = _np(env, "scene", "robot", "data", "root_link_lin_vel_b")
  w = _np(env, "scene", "robot", "data", "root_link_ang_vel_b")
  e_lin = np.sum((c[:, :2] - v[:, :2]) ** 2, 1) + v[:, 2] ** 2
  e_ang = (c[:, 2] - w[:, 2]) ** 2 + np.sum(w[:, :2] ** 2, 1)
  np.testing.assert_allclose(mdp.track_linear_velocity(env, 0.5, "t").numpy(), np.exp(-e_lin / 0.25), rtol=1e-5, atol=1e-12)
  np.testing.assert_allclose(mdp.track_angular_velocity(env, 0.5 ** 0.5, "t").numpy(), np.exp(-e_ang / 0.5), rtol=1e-5, atol=1e-12)


def test_flat_orientation_body_and_root(env):
  """tasks/velocity/mdp/rewards.py:63-85 (body variant projects gravity into the body)."""
  q = _np(env, "scene", "robot", "data", "body_link_quat_w")[:, 3]
  gb = np.array([quat_apply_inverse(_t(qq[None]), _t([0, 0, -1]))[0].numpy() for qq in q])
  std2 = 0.2
  out = mdp.flat_orientation(env, std2 ** 0.5, cfg(body_ids=[3])).numpy()
  np.testing.assert_allclose(out, np.exp(-np.sum(gb[:, :2] ** 2, 1) / std2), rtol=1e-5)
  g = _np(env, "scene", "robot", "data", "projected_gravity_b")
  out = mdp.flat_orientation(env, std2 ** 0.5, cfg(body_ids=[])).numpy()
  np.testing.assert_allclose(out, np.exp(-np.sum(g[:, :2] ** 2, 1) / std2), rtol=1e-5)


def test_penalties(env):
  """rewards.py:88-120 (self collision, body ang vel, angular momentum),
  envs/mdp/rewards.py:56-88 (action rate, joint pos limits)."""
  np.testing.assert_array_equal(mdp.self_collision_cost(env, "self_collision").numpy(),
                                _np(env, "scene", "self_collision", "data", "found")[:, 0])
  w = _np(env, "scene", "robot", "data", "body_link_ang_vel_w")[:, 3]
  np.testing.assert_allclose(mdp.body_angular_velocity_penalty(env, cfg(body_ids=[3])).numpy(),
                             np.sum(w[:, :2] ** 2, 1), rtol=1e-5)
  h = env.scene["angmom"].data.numpy().astype(np.float64)
  np.testing.assert_allclose(mdp.angular_momentum_penalty(env, "angmom").numpy(), np.sum(h ** 2, 1), rtol=1e-5)
  assert env.extras["log"]["Metrics/angular_momentum_mean"] == pytest.approx(np.mean(np.linalg.norm(h, axis=1)), rel=1e-5)
  a, pa = env.action_manager.action.numpy(), env.action_manager.prev_action.numpy()
  np.testing.assert_allclose(mdp.action_rate_l2(env).numpy(), np.sum((a - pa) ** 2, 1), rtol=1e-5)
  q = _np(env, "scene", "robot", "data", "joint_pos")
  lim = _np(env, "scene", "robot", "data", "soft_joint_pos_limits")
  want = np.sum(-np.minimum(q - lim[..., 0], 0) + np.maximum(q - lim[..., 1], 0), 1)
  np.testing.assert_allclose(mdp.joint_pos_limits(env, cfg()).numpy(), want, rtol=1e-5, atol=1e-6)


def test_feet_terms(env):
  """rewards.py:123-288: air time, clearance, slip, soft landing (command-gated)."""
  c = env.command_manager.get_command("t").numpy().astype(np.float64)
  t = _np(env, "scene", "feet", "data", "current_air_time")
  want = np.sum((t > 0.05) & (t < 0.5), 1) * _active(c, 0.5)
  np.testing.assert_allclose(mdp.feet_air_time(env, "feet", 0.05, 0.5, "t", 0.5).numpy(), want)
  z = _np(env, "scene", "robot", "data", "site_pos_w")[..., 2]
  vxy = np.linalg.norm(_np(env, "scene", "robot", "data", "site_lin_vel_w")[..., :2], axis=-1)
  np.testing.assert_allclose(mdp.feet_clearance(env, 0.1, "t", 0.01, cfg(site_ids=[0, 1])).numpy(),
                             np.sum(np.abs(z - 0.1) * vxy, 1) * _active(c, 0.01), rtol=1e-5)
  inc = (_np(env, "scene", "feet", "data", "found") > 0).astype(np.float64)
  np.testing.assert_allclose(mdp.feet_slip(env, "feet", "t", 0.01, cfg(site_ids=[0, 1])).numpy(),
                             np.sum(vxy ** 2 * inc, 1) * _active(c, 0.01), rtol=1e-5)
  fm = np.linalg.norm(_np(env, "scene", "feet", "data", "force"), axis=-1)
  first = env.scene["feet"].first.numpy()
  np.testing.assert_allclose(mdp.soft_landing(env, "feet", "t", 0.05).numpy(),
                             np.sum(fm * first, 1) * _active(c, 0.05), rtol=1e-5)


def test_feet_swing_height_stateful(env):
  """rewards.py:180-229: peak height while airborne, cost at first contact, then reset."""
  term = mdp.feet_swing_height(ns(params={"asset_cfg": ns(site_names=["l", "r"])}), env)
  c = env.command_manager.get_command("t").numpy().astype(np.float64)
  z = _np(env, "scene", "robot", "data", "site_pos_w")[..., 2]
  found = _np(env, "scene", "feet", "data", "found")
  first = env.scene["feet"].first.numpy()
  peak = np.where(found == 0, np.maximum(0.0, z), 0.0)
  want = np.sum(((peak / 0.1) - 1.0) ** 2 * first, 1) * _active(c, 0.01)
  out = term(env, "feet", 0.1, "t", 0.01, cfg(site_ids=[0, 1])).numpy()
  np.testing.assert_allclose(out, want, rtol=1e-5, atol=1e-6)
  np.testing.assert_allclose(term.peak_heights.numpy(), np.where(first, 0.0, peak), rtol=1e-6)


def test_observations(env):
  """envs/mdp/observations.py:24-106, tasks/velocity/mdp/observations.py:17-44."""
  d = env.scene["robot"].data
  np.testing.assert_array_equal(mdp.base_lin_vel(env).numpy(), d.root_link_lin_vel_b.numpy())
  np.testing.assert_array_equal(mdp.projected_gravity(env).numpy(), d.projected_gravity_b.numpy())
  np.testing.assert_allclose(mdp.joint_pos_rel(env, asset_cfg=cfg()).numpy(),
                             (d.joint_pos - d.default_joint_pos).numpy())
  np.testing.assert_allclose(mdp.joint_vel_rel(env, asset_cfg=cfg()).numpy(), d.joint_vel.numpy())
  np.testing.assert_array_equal(mdp.last_action(env).numpy(), env.action_manager.action.numpy())
  np.testing.assert_array_equal(mdp.foot_height(env, cfg(site_ids=[0, 1])).numpy(), d.site_pos_w[:, :, 2].numpy())
  found = env.scene["feet"].data.found.numpy()
  np.testing.assert_array_equal(mdp.foot_contact(env, "feet").numpy(), (found > 0).astype(np.float32))
  f = env.scene["feet"].data.force.numpy().reshape(N, -1).astype(np.float64)
  np.testing.assert_allclose(mdp.foot_contact_forces(env, "feet").numpy(), np.sign(f) * np.log1p(np.abs(f)), rtol=1e-5)


def test_terminations(env):
  """envs/mdp/terminations.py:19-42, tasks/velocity/mdp/terminations.py:13-16."""
  np.testing.assert_array_equal(mdp.time_out(env).numpy(), env.episode_length_buf.numpy() >= 1000)
  g = env.scene["robot"].data.projected_gravity_b.numpy().astype(np.float64)
  lim = math.radians(70.0)
  np.testing.assert_array_equal(mdp.bad_orientation(env, lim).numpy(), np.abs(np.arccos(-g[:, 2])) > lim)
  z = env.scene["robot"].data.root_link_pos_w.numpy()[:, 2]
  np.testing.assert_array_equal(mdp.root_height_below_minimum(env, 0.3).numpy(), z < 0.3)
  nf = env.scene["nonfoot"].data.found.numpy()
  np.testing.assert_array_equal(mdp.illegal_contact(env, "nonfoot").numpy(), np.any(nf > 0, -1))


def test_heading_command_update():
  """tasks/velocity/mdp/velocity_command.py:96-107: heading envs get
  clip(k * wrap(target - heading)); standing envs are zeroed."""
  n = 32
  r = np.random.default_rng(2)
  vel = r.uniform(-1, 1, (n, 3)).astype(np.float32)
  tgt = r.uniform(-np.pi, np.pi, n).astype(np.float32)
  head = r.uniform(-np.pi, np.pi, n).astype(np.float32)
  is_h = r.uniform(size=n) < 0.5
  is_s = r.uniform(size=n) < 0.2
  cmd = object.__new__(mdp.UniformVelocityCommand)
  cmd.cfg = ns(heading_command=True, heading_control_stiffness=0.5, ranges=ns(ang_vel_z=(-0.5, 0.5)))
  cmd.vel_command_b = _t(vel.copy())
  cmd.heading_target = _t(tgt)
  cmd.is_heading_env = torch.as_tensor(is_h)
  cmd.is_standing_env = torch.as_tensor(is_s)
  cmd.heading_error = torch.zeros(n)
  cmd.robot = ns(data=ns(heading_w=_t(head)))
  cmd._update_command()
  err = (tgt.astype(np.float64) - head + np.pi) % (2 * np.pi) - np.pi
  want = vel.astype(np.float64).copy()
  want[is_h, 2] = np.clip(0.5 * err[is_h], -0.5, 0.5)
  want[is_s] = 0.0
  np.testing.assert_allclose(cmd.vel_command_b.numpy(), want, atol=1e-6)


def test_air_time_tracking_state_machine():
  """sensor/contact_sensor.py:327-367 (air/contact timers), :260-280 (first contact/air)."""
  from mjlab_amd.scene import ContactSensor
  n, s, T, dt = 6, 2, 30, 0.005
  r = np.random.default_rng(3)
  found = np.zeros((T, n, s), np.float32)
  for i in range(n):
    for j in range(s):
      state, k = int(r.integers(0, 2)), 0
      while k < T:
        run = int(r.integers(1, 7))
        found[k:k + run, i, j] = state
        state, k = 1 - state, k + run
  sens = object.__new__(ContactSensor)
  z = lambda: torch.zeros(n, s)
  sens._air = dict(current_air_time=z(), last_air_time=z(), current_contact_time=z(),
                   last_contact_time=z(), last_time=torch.zeros(n))
  sens._fields = ("found",)
  cur = {}
  sens._extract = lambda: ns(found=cur["f"])
  sens._data = ns()
  # restated in fp32, like the reference's tensors (first-contact thresholds sit at dt)
  f32 = np.float32
  ca = np.zeros((n, s), f32); la = np.zeros((n, s), f32); cc = np.zeros((n, s), f32)
  lc = np.zeros((n, s), f32)
  last_t = np.zeros(n, f32)
  for k in range(T):
    t = f32((k + 1) * dt)
    cur["f"] = torch.as_tensor(found[k])
    sens._data.time = torch.full((n,), float(t), dtype=torch.float32)
    sens.update(dt)
    el = (t - last_t)[:, None]
    contact = found[k] > 0
    fc = (ca > 0) & contact
    fd = (cc > 0) & ~contact
    la = np.where(fc, ca + el, la).astype(f32)
    ca = np.where(~contact, ca + el, f32(0)).astype(f32)
    lc = np.where(fd, cc + el, lc).astype(f32)
    cc = np.where(contact, cc + el, f32(0)).astype(f32)
    last_t[:] = t
    a = sens._air
    np.testing.assert_allclose(a["current_air_time"].numpy(), ca, atol=1e-6)
    np.testing.assert_allclose(a["last_air_time"].numpy(), la, atol=1e-6)
    np.testing.assert_allclose(a["current_contact_time"].numpy(), cc, atol=1e-6)
    np.testing.assert_allclose(a["last_contact_time"].numpy(), lc, atol=1e-6)
    np.testing.assert_array_equal(sens.compute_first_contact(dt).numpy(), (cc > 0) & (cc < f32(dt + 1e-8)))
    np.testing.assert_array_equal(sens.compute_first_air(dt).numpy(), (ca > 0) & (ca < f32(dt + 1e-8)))


def test_math_helpers():
  """utils/lab_api/math.py: quat_apply(_inverse) :629-670, yaw_quat :566-588,
  wrap_to_pi :102-125, matrix_from_quat / quat_from_matrix round trip :166-372."""
  q = _t(_unit(64))
  v = _t(rng.standard_normal((64, 3)))
  R = matrix_from_quat(q).numpy()
  np.testing.assert_allclose(quat_apply(q, v).numpy(), np.einsum("nij,nj->ni", R, v.numpy()), atol=1e-5)
  np.testing.assert_allclose(quat_apply_inverse(q, quat_apply(q, v)).numpy(), v.numpy(), atol=1e-5)
  # the round trip in float64: in float32 a component near 0 carries ~sqrt(eps32) error
  q2 = quat_from_matrix(matrix_from_quat(q.double())).numpy()
  sign = np.sign(np.sum(q2 * q.numpy(), -1, keepdims=True))
  np.testing.assert_allclose(q2 * sign, q.numpy(), atol=1e-6)
  qq = quat_mul(q, _t(_unit(64)))
  np.testing.assert_allclose(np.linalg.norm(qq.numpy(), axis=-1), 1.0, atol=1e-5)
  y = yaw_quat(q).numpy()
  assert np.allclose(y[:, 1:3], 0.0, atol=1e-6)
  np.testing.assert_allclose(np.linalg.norm(y, axis=-1), 1.0, atol=1e-5)
  a = _t(rng.uniform(-20, 20, 200))
  w = wrap_to_pi(a).numpy()
  assert np.all(w >= -np.pi - 1e-6) and np.all(w <= np.pi + 1e-6)
  np.testing.assert_allclose(np.cos(w), np.cos(a.numpy()), atol=1e-4)
  e = _t(rng.uniform(-np.pi, np.pi, (32, 3)))
  qe = quat_from_euler_xyz(e[:, 0], e[:, 1], e[:, 2])
  Rz = lambda t: np.array([[np.cos(t), -np.sin(t), 0], [np.sin(t), np.cos(t), 0], [0, 0, 1]])
  Ry = lambda t: np.array([[np.cos(t), 0, np.sin(t)], [0, 1, 0], [-np.sin(t), 0, np.cos(t)]])
  Rx = lambda t: np.array([[1, 0, 0], [0, np.cos(t), -np.sin(t)], [0, np.sin(t), np.cos(t)]])
  for i in range(32):
    r, p, yw = e[i].numpy().astype(np.float64)
    np.testing.assert_allclose(matrix_from_quat(qe[i:i + 1])[0].numpy(), Rz(yw) @ Ry(p) @ Rx(r), atol=1e-5)


def test_resolve_matching_names():
  """utils/lab_api/string.py:178-260: full-match, natural order unless preserve_order,
  error on unmatched keys."""
  names = ["left_hip", "right_hip", "left_knee", "right_knee"]
  with pytest.raises(ValueError):  # one name matched by two keys
    resolve_matching_names([".*_knee", "left_.*"], names)
  idx, out = resolve_matching_names([".*_knee"], names)
  assert (idx, out) == ([2, 3], ["left_knee", "right_knee"])
  idx, out = resolve_matching_names(["right_.*", "left_.*"], names, preserve_order=True)
  assert out == ["right_hip", "right_knee", "left_hip", "left_knee"]
  with pytest.raises(ValueError):
    resolve_matching_names(["foot"], names)
  idx, nm, vals = resolve_matching_names_values({".*_hip": 1.0, ".*": 2.0}, names)
  assert vals == [1.0, 1.0, 2.0, 2.0]
