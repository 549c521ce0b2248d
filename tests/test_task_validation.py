"""Task-descriptor validation at the C ABI: mjx_task_create /
mjx_track_create check every index the fused manager kernels dereference against the sizes the
descriptor declares, and every term / command kind against the buffers and observation layout
it reads, before anything reaches the device.  A mismatch is a nonzero status with a message in
mjx_task_last_error / mjx_track_last_error -- not a GPU fault (round 5: the twist-command read
on the jump task's [nworld, 1] command faulted the device).

No GPU: validation runs before the first HIP call, so a consistent descriptor gets as far as
"hipMalloc failed" here (that message is the proof it passed validation)."""

import ctypes
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "mjlab-1_amd", "mjlab_amd", "libmjx355.so")

# a G1-shaped velocity task: 29 joints, 2 feet, free joint first
NQ, NV, NU, NBODY, NSITE, NSD, NJ, NF = 36, 35, 29, 31, 6, 40, 29, 2
MJX_CMD_TWIST, MJX_CMD_JUMP = 0, 1


@pytest.fixture(scope="module")
def lib():
  if not os.path.exists(LIB):
    pytest.skip("libmjx355.so not built (run __graft_entry__.build())")
  L = ctypes.CDLL(LIB)
  for f in ("mjx_task_last_error", "mjx_track_last_error"):
    getattr(L, f).restype = ctypes.c_char_p
  return L


def _fill_pointers(d):
  """Every pointer field of the descriptor set to a dummy non-null address (never read on the
  host; the create call fails at hipMalloc on a GPU-less host after validation)."""
  for name, typ in d._fields_:
    if isinstance(typ, type) and issubclass(typ, ctypes._Pointer):
      setattr(d, name, ctypes.cast(ctypes.c_void_p(0x1000), typ))


def _velocity_desc():
  from mjlab_amd.fused import TaskDesc
  d = TaskDesc()
  _fill_pointers(d)
  d.nworld, d.nq, d.nv, d.nu, d.nsensordata, d.nbody, d.nsite = 16, NQ, NV, NU, NSD, NBODY, NSITE
  d.root_body, d.free_q_adr, d.free_v_adr, d.njoint = 1, 0, 0, NJ
  for j in range(NJ):
    d.joint_q_adr[j], d.joint_v_adr[j], d.ctrl_of_action[j], d.target_of_action[j] = 7 + j, 6 + j, j, j
    d.act_ctrl[j] = j
  d.nfeet = NF
  for s in range(NF):
    d.foot_site[s], d.foot_site_body[s], d.feet_found_adr[s], d.feet_force_adr[s] = s, 6 + 6 * s, 20 + s, 22 + 3 * s
  d.imu_lin_vel_adr, d.imu_ang_vel_adr, d.angmom_adr, d.selfcol_found_adr = 0, 3, 6, 9
  d.nillegal, d.orient_body = 0, 1
  d.step_dt, d.episode_length_s, d.max_episode_length = 0.02, 20.0, 1000
  kinds = [0, 1, 2, 4, 5, 6, 7, 8, 11, 13]
  d.nreward = len(kinds)
  for k, kind in enumerate(kinds):
    d.reward_kind[k], d.reward_weight[k], d.reward_p0[k] = kind, 1.0, 0.5
  d.ntermination = 2
  d.termination_kind[0], d.termination_is_timeout[0] = 0, 1
  d.termination_kind[1], d.termination_p0[1] = 1, 1.2
  d.command_kind = MJX_CMD_TWIST
  d.npolicy = 9 + 3 * NJ + 3
  d.critic_extras = 1
  d.ncritic = d.npolicy + 6 * NF
  return d


def _create(L, d):
  out = ctypes.c_void_p()
  rc = L.mjx_task_create(ctypes.byref(d), ctypes.byref(out))
  return rc, L.mjx_task_last_error().decode()


def test_consistent_descriptor_passes_validation(lib):
  rc, msg = _create(lib, _velocity_desc())
  # validation passed: the call reached the device allocation (no GPU here), or succeeded
  assert rc == 0 or "hipMalloc" in msg or "upload" in msg, msg


@pytest.mark.parametrize("mutate, needle", [
  # the round-5 fault: a twist-reading reward on the jump command ([nworld, 1])
  (lambda d: setattr(d, "command_kind", MJX_CMD_JUMP), "twist command"),
  (lambda d: d.joint_q_adr.__setitem__(3, NQ), "qpos address"),
  (lambda d: d.joint_v_adr.__setitem__(0, -1), "qvel address"),
  (lambda d: d.ctrl_of_action.__setitem__(5, NU), "ctrl index"),
  (lambda d: d.target_of_action.__setitem__(5, NJ), "joint_pos_target"),
  (lambda d: d.foot_site.__setitem__(1, NSITE), "site"),
  (lambda d: d.feet_force_adr.__setitem__(0, NSD - 2), "force sensor"),
  (lambda d: setattr(d, "imu_ang_vel_adr", NSD - 1), "imu"),
  (lambda d: setattr(d, "root_body", NBODY), "root_body"),
  (lambda d: setattr(d, "free_q_adr", NQ - 3), "free joint qpos"),
  (lambda d: setattr(d, "angmom_adr", -1), "angmom_adr"),
  (lambda d: d.reward_kind.__setitem__(2, 99), "unknown kind"),
  (lambda d: d.termination_kind.__setitem__(1, 7), "unknown kind"),
  (lambda d: d.termination_kind.__setitem__(1, 2), "illegal_contact"),
  (lambda d: setattr(d, "ncritic", 9 + 3 * NJ + 3), "observation widths"),
  (lambda d: setattr(d, "npolicy", 9 + 3 * NJ), "observation widths"),
  (lambda d: setattr(d, "command_kind", 5), "command_kind"),
  (lambda d: setattr(d, "qpos", None), "required buffer"),
  (lambda d: setattr(d, "cur_air", None), "foot buffer"),
  (lambda d: setattr(d, "njoint", 65), "capacities"),
])
def test_mismatched_descriptor_is_an_error(lib, mutate, needle):
  d = _velocity_desc()
  mutate(d)
  rc, msg = _create(lib, d)
  assert rc != 0
  assert needle in msg, msg
  assert "hipMalloc" not in msg


def test_jump_layout_checked(lib):
  """The jump descriptor: twist-free terms, the jump observation layout, its state buffers."""
  d = _velocity_desc()
  d.command_kind = MJX_CMD_JUMP
  kinds = [2, 6, 7, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23]
  d.nreward = len(kinds)
  for k, kind in enumerate(kinds):
    d.reward_kind[k], d.reward_weight[k] = kind, 1.0
  d.npolicy = 9 + 3 * NJ + 3 + 2 * NF
  d.ncritic = d.npolicy + 4 * NF
  rc, msg = _create(lib, d)
  assert rc == 0 or "hipMalloc" in msg or "upload" in msg, msg
  d.ncritic = d.npolicy + 6 * NF  # the velocity critic extras: wrong for the jump layout
  rc, msg = _create(lib, d)
  assert rc != 0 and "jump task layout" in msg, msg
  d.ncritic = d.npolicy + 4 * NF
  d.landing_timer = None
  rc, msg = _create(lib, d)
  assert rc != 0 and "landing_timer" in msg, msg


def _track_desc():
  from mjlab_amd.fused_tracking import TrackDesc
  d = TrackDesc()
  _fill_pointers(d)
  nmb = 14
  d.nworld, d.nq, d.nv, d.nu, d.nsensordata, d.nbody = 16, NQ, NV, NU, NSD, NBODY
  d.root_body, d.free_q_adr, d.free_v_adr, d.njoint = 1, 0, 0, NJ
  for j in range(NJ):
    d.joint_q_adr[j], d.joint_v_adr[j], d.ctrl_of_action[j], d.target_of_action[j] = 7 + j, 6 + j, j, j
  d.nframe, d.nmb = 100, nmb
  for k in range(nmb):
    d.robot_body[k] = 1 + k
  d.anchor_motion, d.anchor_body = 3, 4
  d.step_dt, d.episode_length_s, d.max_episode_length = 0.02, 10.0, 500
  d.nreward = 3
  d.reward_kind[0], d.reward_kind[1], d.reward_kind[2] = 0, 2, 8
  d.reward_bodies[1] = (1 << nmb) - 1
  d.ntermination = 2
  d.termination_kind[0], d.termination_kind[1] = 0, 3
  d.termination_bodies[1] = 0b11
  d.selfcol_found_adr, d.imu_lin_vel_adr, d.imu_ang_vel_adr = 9, 0, 3
  d.sampling_mode, d.bin_count, d.kernel_size = 2, 50, 3
  d.policy_anchor_pos = d.policy_lin_vel = 1
  d.npolicy = 5 * NJ + 9 + 6
  d.ncritic = 5 * NJ + 9 * nmb + 15
  return d


def test_tracking_descriptor_validation(lib):
  out = ctypes.c_void_p()

  def create(d):
    rc = lib.mjx_track_create(ctypes.byref(d), ctypes.byref(out))
    return rc, lib.mjx_track_last_error().decode()

  rc, msg = create(_track_desc())
  assert rc == 0 or "hipMalloc" in msg or "upload" in msg, msg
  for mutate, needle in [
    (lambda d: d.robot_body.__setitem__(2, NBODY), "model body"),
    (lambda d: setattr(d, "anchor_motion", 14), "anchor_motion"),
    (lambda d: d.reward_bodies.__setitem__(1, 1 << 20), "body mask"),
    (lambda d: d.reward_kind.__setitem__(0, 12), "unknown kind"),
    (lambda d: setattr(d, "selfcol_found_adr", -1), "selfcol_found_adr"),
    (lambda d: d.joint_q_adr.__setitem__(0, NQ), "qpos address"),
    (lambda d: setattr(d, "encoder_bias", None), "required buffer"),
    (lambda d: setattr(d, "npolicy", 5 * NJ + 9), "observation sizes"),
  ]:
    d = _track_desc()
    mutate(d)
    rc, msg = create(d)
    assert rc != 0 and needle in msg, (needle, msg)
