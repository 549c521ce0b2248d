"""Runtime scene: entities (index tensors + world-frame views) and sensors over the
engine's device fields.

Mirrors `src/mjlab/entity/entity.py:390-825`, `src/mjlab/entity/data.py:20-533`,
`src/mjlab/sensor/builtin_sensor.py`, `src/mjlab/sensor/contact_sensor.py:199-367` and
`src/mjlab/scene/scene.py:29-198`.  The scene is assembled at env construction
from a `SceneCfg` (entities, terrain, sensors) by this build's MJCF compiler, and the runtime
views bind to the compiled model's name tables.
"""

from __future__ import annotations

import re
from dataclasses import dataclass, field

import numpy as np
import torch

from .managers import resolve_matching_names
from .math_utils import quat_apply, quat_apply_inverse

OBJ_SITE = 6


def compute_velocity_from_cvel(pos, subtree_com, cvel):
  """cvel = [ang; lin at subtree_com(root)] -> [lin at pos; ang] (entity/data.py:20-31)."""
  lin_c = cvel[..., 3:6]
  ang = cvel[..., 0:3]
  lin = lin_c - torch.cross(ang, subtree_com - pos, dim=-1)
  return torch.cat([lin, ang], dim=-1)


@dataclass
class EntityIndexing:
  root_body_id: int
  body_ids: torch.Tensor
  geom_ids: torch.Tensor
  site_ids: torch.Tensor
  ctrl_ids: torch.Tensor
  joint_q_adr: torch.Tensor
  joint_v_adr: torch.Tensor
  free_joint_q_adr: torch.Tensor
  free_joint_v_adr: torch.Tensor
  site_body_ids: torch.Tensor
  joint_ids: torch.Tensor | None = None


class EntityData:
  """World-frame reads and state writes for one entity (entity/data.py)."""

  def __init__(self, indexing, data, model, device, num_envs, default_root_state,
               default_joint_pos, default_joint_vel, joint_pos_limits, soft_limits):
    self.indexing = indexing
    self.data = data
    self.model = model
    self.device = device
    self.default_root_state = default_root_state
    self.default_joint_pos = default_joint_pos
    self.default_joint_vel = default_joint_vel
    self.default_joint_pos_limits = joint_pos_limits.clone()
    self.joint_pos_limits = joint_pos_limits
    self.soft_joint_pos_limits = soft_limits
    nj = default_joint_pos.shape[1]
    self.joint_pos_target = torch.zeros(num_envs, nj, device=device)
    self.joint_vel_target = torch.zeros(num_envs, nj, device=device)
    self.joint_effort_target = torch.zeros(num_envs, nj, device=device)
    self.encoder_bias = torch.zeros(num_envs, nj, device=device)
    self.gravity_vec_w = torch.tensor([0.0, 0.0, -1.0], device=device).repeat(num_envs, 1)
    self.forward_vec_b = torch.tensor([1.0, 0.0, 0.0], device=device).repeat(num_envs, 1)
    self.is_fixed_base = False
    self.is_articulated = nj > 0
    self.is_actuated = len(indexing.ctrl_ids) > 0

  # ---------------------------------------------------------------- writes
  def _env(self, env_ids):
    if env_ids is None:
      return slice(None)
    if isinstance(env_ids, torch.Tensor):
      return env_ids[:, None]
    return env_ids

  def write_root_state(self, root_state, env_ids=None):
    self.write_root_pose(root_state[:, :7], env_ids)
    self.write_root_velocity(root_state[:, 7:], env_ids)

  def write_root_pose(self, pose, env_ids=None):
    e = self._env(env_ids)
    self.data.qpos[e, self.indexing.free_joint_q_adr] = pose

  def write_root_velocity(self, velocity, env_ids=None):
    """World-frame [lin, ang] -> qvel with angular in body frame via the qpos quat
    (entity/data.py:99-110)."""
    e = self._env(env_ids)
    quat_w = self.data.qpos[e, self.indexing.free_joint_q_adr[3:7]]
    ang_b = quat_apply_inverse(quat_w, velocity[:, 3:])
    self.data.qvel[e, self.indexing.free_joint_v_adr] = torch.cat([velocity[:, :3], ang_b], -1)

  def write_joint_state(self, position, velocity, joint_ids=None, env_ids=None):
    self.write_joint_position(position, joint_ids, env_ids)
    self.write_joint_velocity(velocity, joint_ids, env_ids)

  def write_joint_position(self, position, joint_ids=None, env_ids=None):
    e = self._env(env_ids)
    jid = joint_ids if joint_ids is not None else slice(None)
    self.data.qpos[e, self.indexing.joint_q_adr[jid]] = position

  def write_joint_velocity(self, velocity, joint_ids=None, env_ids=None):
    e = self._env(env_ids)
    jid = joint_ids if joint_ids is not None else slice(None)
    self.data.qvel[e, self.indexing.joint_v_adr[jid]] = velocity

  def write_ctrl(self, ctrl, ctrl_ids=None, env_ids=None):
    e = self._env(env_ids)
    cid = ctrl_ids if ctrl_ids is not None else slice(None)
    self.data.ctrl[e, self.indexing.ctrl_ids[cid]] = ctrl

  def write_external_wrench(self, force, torque, body_ids=None, env_ids=None):
    e = self._env(env_ids)
    b = self.indexing.body_ids[body_ids if body_ids is not None else slice(None)]
    if force is not None:
      self.data.xfrc_applied[e, b, 0:3] = force
    if torque is not None:
      self.data.xfrc_applied[e, b, 3:6] = torque

  # ---------------------------------------------------------------- masked (sync-free) writes
  def write_root_pose_masked(self, pose, mask):
    q = self.data.qpos
    adr = self.indexing.free_joint_q_adr
    q[:, adr] = torch.where(mask.unsqueeze(1), pose, q[:, adr])

  def write_root_velocity_masked(self, velocity, mask):
    q = self.data.qpos
    quat_w = q[:, self.indexing.free_joint_q_adr[3:7]]
    ang_b = quat_apply_inverse(quat_w, velocity[:, 3:])
    v = self.data.qvel
    adr = self.indexing.free_joint_v_adr
    v[:, adr] = torch.where(mask.unsqueeze(1), torch.cat([velocity[:, :3], ang_b], -1), v[:, adr])

  def write_joint_state_masked(self, position, velocity, mask, joint_ids=None):
    jid = joint_ids if joint_ids is not None else slice(None)
    qa = self.indexing.joint_q_adr[jid]
    va = self.indexing.joint_v_adr[jid]
    m = mask.unsqueeze(1)
    self.data.qpos[:, qa] = torch.where(m, position, self.data.qpos[:, qa])
    self.data.qvel[:, va] = torch.where(m, velocity, self.data.qvel[:, va])

  def clear_state_masked(self, mask):
    m = mask.unsqueeze(1)
    for t in (self.joint_pos_target, self.joint_vel_target, self.joint_effort_target):
      t.masked_fill_(m, 0.0)

  def clear_state(self, env_ids=None):
    e = slice(None) if env_ids is None else env_ids
    self.joint_pos_target[e] = 0.0
    self.joint_vel_target[e] = 0.0
    self.joint_effort_target[e] = 0.0

  # ---------------------------------------------------------------- root reads
  @property
  def root_link_pos_w(self):
    return self.data.xpos[:, self.indexing.root_body_id]

  @property
  def root_link_quat_w(self):
    return self.data.xquat[:, self.indexing.root_body_id]

  @property
  def root_link_pose_w(self):
    return torch.cat([self.root_link_pos_w, self.root_link_quat_w], dim=-1)

  @property
  def root_link_vel_w(self):
    r = self.indexing.root_body_id
    return compute_velocity_from_cvel(self.data.xpos[:, r], self.data.subtree_com[:, r],
                                      self.data.cvel[:, r])

  @property
  def root_link_lin_vel_w(self):
    return self.root_link_vel_w[:, 0:3]

  @property
  def root_link_ang_vel_w(self):
    return self.data.cvel[:, self.indexing.root_body_id, 0:3]

  @property
  def root_com_pos_w(self):
    return self.data.xipos[:, self.indexing.root_body_id]

  @property
  def root_com_vel_w(self):
    r = self.indexing.root_body_id
    return compute_velocity_from_cvel(self.data.xipos[:, r], self.data.subtree_com[:, r],
                                      self.data.cvel[:, r])

  @property
  def root_link_lin_vel_b(self):
    return quat_apply_inverse(self.root_link_quat_w, self.root_link_lin_vel_w)

  @property
  def root_link_ang_vel_b(self):
    return quat_apply_inverse(self.root_link_quat_w, self.root_link_ang_vel_w)

  @property
  def projected_gravity_b(self):
    return quat_apply_inverse(self.root_link_quat_w, self.gravity_vec_w)

  @property
  def heading_w(self):
    f = quat_apply(self.root_link_quat_w, self.forward_vec_b)
    return torch.atan2(f[:, 1], f[:, 0])

  # ---------------------------------------------------------------- bodies / sites
  @property
  def body_link_pos_w(self):
    return self.data.xpos[:, self.indexing.body_ids]

  @property
  def body_link_quat_w(self):
    return self.data.xquat[:, self.indexing.body_ids]

  @property
  def body_link_pose_w(self):
    return torch.cat([self.body_link_pos_w, self.body_link_quat_w], dim=-1)

  @property
  def body_link_vel_w(self):
    sc = self.data.subtree_com[:, self.indexing.root_body_id].unsqueeze(1)
    return compute_velocity_from_cvel(self.data.xpos[:, self.indexing.body_ids], sc,
                                      self.data.cvel[:, self.indexing.body_ids])

  @property
  def body_link_lin_vel_w(self):
    return self.body_link_vel_w[..., 0:3]

  @property
  def body_link_ang_vel_w(self):
    return self.data.cvel[:, self.indexing.body_ids, 0:3]

  @property
  def body_com_pos_w(self):
    return self.data.xipos[:, self.indexing.body_ids]

  @property
  def site_pos_w(self):
    return self.data.site_xpos[:, self.indexing.site_ids]

  @property
  def site_vel_w(self):
    sc = self.data.subtree_com[:, self.indexing.root_body_id].unsqueeze(1)
    return compute_velocity_from_cvel(self.data.site_xpos[:, self.indexing.site_ids], sc,
                                      self.data.cvel[:, self.indexing.site_body_ids])

  @property
  def site_lin_vel_w(self):
    return self.site_vel_w[..., 0:3]

  @property
  def geom_pos_w(self):
    return self.data.geom_xpos[:, self.indexing.geom_ids]

  # ---------------------------------------------------------------- joints
  @property
  def joint_pos(self):
    return self.data.qpos[:, self.indexing.joint_q_adr]

  @property
  def joint_pos_biased(self):
    return self.joint_pos + self.encoder_bias

  @property
  def joint_vel(self):
    return self.data.qvel[:, self.indexing.joint_v_adr]

  @property
  def joint_acc(self):
    return self.data.qacc[:, self.indexing.joint_v_adr]

  @property
  def actuator_force(self):
    return self.data.actuator_force[:, self.indexing.ctrl_ids]


class Entity:
  """One attached MJCF entity (prefix '<name>/') with builtin position actuators."""

  def __init__(self, name: str, mj_model, soft_joint_pos_limit_factor: float = 0.9,
               init_lin_vel=(0.0, 0.0, 0.0), init_ang_vel=(0.0, 0.0, 0.0)):
    self.name = name
    self._m = mj_model
    self._prefix = f"{name}/"
    self._soft = soft_joint_pos_limit_factor
    self._init_vel = tuple(init_lin_vel) + tuple(init_ang_vel)
    m = mj_model
    strip = lambda n: n[len(self._prefix):]
    self._body_gid = [i for i, n in enumerate(m.names["body"]) if n.startswith(self._prefix)]
    self._geom_gid = [i for i, n in enumerate(m.names["geom"]) if n.startswith(self._prefix)]
    self._site_gid = [i for i, n in enumerate(m.names["site"]) if n.startswith(self._prefix)]
    self._act_gid = [i for i, n in enumerate(m.names["actuator"]) if n.startswith(self._prefix)]
    jall = [i for i, n in enumerate(m.names["joint"]) if n.startswith(self._prefix)]
    self._free_jid = [j for j in jall if m.jnt_type[j] == 0]
    self._jnt_gid = [j for j in jall if m.jnt_type[j] != 0]
    self.body_names = tuple(strip(m.names["body"][i]) for i in self._body_gid)
    self.geom_names = tuple(strip(m.names["geom"][i]) for i in self._geom_gid)
    self.site_names = tuple(strip(m.names["site"][i]) for i in self._site_gid)
    self.joint_names = tuple(strip(m.names["joint"][j]) for j in self._jnt_gid)
    self.actuator_names = tuple(strip(m.names["actuator"][i]) for i in self._act_gid)
    self.is_fixed_base = len(self._free_jid) == 0
    self.is_articulated = len(self._jnt_gid) > 0
    self.is_actuated = len(self._act_gid) > 0
    # actuator -> entity-local joint index (BuiltinActuatorGroup, actuator/builtin_group.py)
    self._act_joint_local = [self._jnt_gid.index(int(m.actuator_trnid[a])) for a in self._act_gid]

  # name resolution (natural order)
  def find_joints(self, keys, joint_subset=None, preserve_order=False):
    return resolve_matching_names(keys, joint_subset or self.joint_names, preserve_order)

  def find_bodies(self, keys, preserve_order=False):
    return resolve_matching_names(keys, self.body_names, preserve_order)

  def find_geoms(self, keys, preserve_order=False):
    return resolve_matching_names(keys, self.geom_names, preserve_order)

  def find_sites(self, keys, preserve_order=False):
    return resolve_matching_names(keys, self.site_names, preserve_order)

  def find_actuators(self, keys, preserve_order=False):
    return resolve_matching_names(keys, self.actuator_names, preserve_order)

  def find_joints_by_actuator_names(self, actuator_name_keys):
    _, act_names = self.find_actuators(actuator_name_keys)
    actuated = set(act_names)
    names = [n for n in self.joint_names if n in actuated]
    return [self.joint_names.index(n) for n in names], names

  def initialize(self, mj_model, model, data, device: str):
    m = mj_model
    dev = device
    n = data.qpos.shape[0]
    t = lambda x: torch.as_tensor(np.asarray(x), dtype=torch.long, device=dev)
    root = self._body_gid[0]
    fq = (list(range(m.jnt_qposadr[self._free_jid[0]], m.jnt_qposadr[self._free_jid[0]] + 7))
          if self._free_jid else [])
    fv = (list(range(m.jnt_dofadr[self._free_jid[0]], m.jnt_dofadr[self._free_jid[0]] + 6))
          if self._free_jid else [])
    self.indexing = EntityIndexing(
      root_body_id=root, body_ids=t(self._body_gid), geom_ids=t(self._geom_gid),
      site_ids=t(self._site_gid), ctrl_ids=t(self._act_gid),
      joint_q_adr=t([m.jnt_qposadr[j] for j in self._jnt_gid]),
      joint_v_adr=t([m.jnt_dofadr[j] for j in self._jnt_gid]),
      free_joint_q_adr=t(fq), free_joint_v_adr=t(fv),
      site_body_ids=t([m.site_bodyid[s] for s in self._site_gid]),
      joint_ids=t(self._jnt_gid))
    key = np.asarray(m.key_qpos)
    root_state = np.zeros(13)
    if fq:
      root_state[:7] = key[fq]
      root_state[7:] = self._init_vel
    drs = torch.tensor(root_state, dtype=torch.float32, device=dev).repeat(n, 1)
    djp = torch.tensor(key[[m.jnt_qposadr[j] for j in self._jnt_gid]], dtype=torch.float32,
                       device=dev).repeat(n, 1)
    djv = torch.zeros_like(djp)
    rng = torch.tensor(np.asarray(m.jnt_range)[self._jnt_gid], dtype=torch.float32,
                       device=dev).repeat(n, 1, 1)
    mean = 0.5 * (rng[..., 0] + rng[..., 1])
    half = 0.5 * (rng[..., 1] - rng[..., 0]) * self._soft
    soft = torch.stack([mean - half, mean + half], dim=-1)
    self._data = EntityData(self.indexing, data, model, dev, n, drs, djp, djv, rng, soft)
    self._act_joint_local_t = t(self._act_joint_local)

  @property
  def data(self) -> EntityData:
    return self._data

  @property
  def num_joints(self):
    return len(self.joint_names)

  # writes (entity.py:520-640)
  def write_root_state_to_sim(self, root_state, env_ids=None):
    self._data.write_root_state(root_state, env_ids)

  def write_root_link_pose_to_sim(self, pose, env_ids=None):
    self._data.write_root_pose(pose, env_ids)

  def write_root_link_velocity_to_sim(self, velocity, env_ids=None):
    self._data.write_root_velocity(velocity, env_ids)

  def write_joint_state_to_sim(self, position, velocity, joint_ids=None, env_ids=None):
    self._data.write_joint_state(position, velocity, joint_ids, env_ids)

  def write_joint_position_to_sim(self, position, joint_ids=None, env_ids=None):
    self._data.write_joint_position(position, joint_ids, env_ids)

  def write_joint_velocity_to_sim(self, velocity, joint_ids=None, env_ids=None):
    self._data.write_joint_velocity(velocity, joint_ids, env_ids)

  def write_external_wrench_to_sim(self, force, torque, env_ids=None, body_ids=None):
    self._data.write_external_wrench(force, torque, body_ids, env_ids)

  def set_joint_position_target(self, position, joint_ids=None, env_ids=None):
    e = slice(None) if env_ids is None else env_ids
    j = slice(None) if joint_ids is None else joint_ids
    self._data.joint_pos_target[e, j] = position

  def set_joint_velocity_target(self, velocity, joint_ids=None, env_ids=None):
    e = slice(None) if env_ids is None else env_ids
    j = slice(None) if joint_ids is None else joint_ids
    self._data.joint_vel_target[e, j] = velocity

  def set_joint_effort_target(self, effort, joint_ids=None, env_ids=None):
    e = slice(None) if env_ids is None else env_ids
    j = slice(None) if joint_ids is None else joint_ids
    self._data.joint_effort_target[e, j] = effort

  def write_data_to_sim(self):
    """BuiltinActuatorGroup.apply_controls: ctrl[:, ctrl_ids] = target[:, joint_ids]."""
    if self.is_actuated:
      self._data.data.ctrl[:, self.indexing.ctrl_ids] = \
        self._data.joint_pos_target[:, self._act_joint_local_t]

  def update(self, dt: float):
    pass

  def reset(self, env_ids=None):
    self._data.clear_state(env_ids)

  def reset_masked(self, mask):
    self._data.clear_state_masked(mask)


class BuiltinSensor:
  """View into sensordata for one MJCF sensor (sensor/builtin_sensor.py:327-335)."""

  def __init__(self, name: str, adr: int, dim: int):
    self.name, self._adr, self._dim = name, adr, dim
    self._view = None

  def initialize(self, data):
    self._view = data.sensordata[:, self._adr: self._adr + self._dim]

  @property
  def data(self) -> torch.Tensor:
    return self._view

  def update(self, dt):
    pass

  def reset(self, env_ids=None):
    pass

  def reset_masked(self, mask):
    pass


@dataclass
class ContactData:
  found: torch.Tensor | None = None
  force: torch.Tensor | None = None
  torque: torch.Tensor | None = None
  dist: torch.Tensor | None = None
  pos: torch.Tensor | None = None
  normal: torch.Tensor | None = None
  tangent: torch.Tensor | None = None
  current_air_time: torch.Tensor | None = None
  last_air_time: torch.Tensor | None = None
  current_contact_time: torch.Tensor | None = None
  last_contact_time: torch.Tensor | None = None


_FIELD_DIM = {"found": 1, "force": 3, "torque": 3, "dist": 1, "pos": 3, "normal": 3, "tangent": 3}


class ContactSensor:
  """mjSENS_CONTACT group expanded per primary x field (sensor/contact_sensor.py)."""

  # set while a fused env step has handed the air-time buffers to the engine
  # (mjx_sim_track_air_time): phase C then updates them every substep
  engine_owned = False

  def __init__(self, name: str, slots: list[tuple[str, str, int, int]], fields, num_slots: int,
               track_air_time: bool):
    self.name = name
    self._slots = slots  # (primary, field, adr, dim)
    self._fields = tuple(fields)
    self._num_slots = num_slots
    self._track = track_air_time
    self._data = None
    self._air = None
    n_primary = len({s[0] for s in slots})
    self._n_primary = n_primary

  def initialize(self, data, device):
    self._data = data
    self._views = {f: [] for f in self._fields}
    for prim, f, adr, dim in self._slots:
      self._views[f].append(data.sensordata[:, adr: adr + dim])
    if self._track:
      n = data.time.shape[0]
      z = lambda: torch.zeros(n, self._n_primary, device=device)
      self._air = dict(current_air_time=z(), last_air_time=z(), current_contact_time=z(),
                       last_contact_time=z(), last_time=torch.zeros(n, device=device))

  def _extract(self) -> ContactData:
    out = ContactData()
    for f, views in self._views.items():
      d = _FIELD_DIM[f]
      chunks = [v.reshape(v.shape[0], self._num_slots, d) for v in views]
      cat = torch.cat(chunks, dim=1)
      if d == 1:
        cat = cat.squeeze(-1)
      setattr(out, f, cat)
    return out

  @property
  def data(self) -> ContactData:
    out = self._extract()
    if self._air is not None:
      for k in ("current_air_time", "last_air_time", "current_contact_time", "last_contact_time"):
        setattr(out, k, self._air[k])
    return out

  def reset(self, env_ids=None):
    if self._air is None:
      return
    e = slice(None) if env_ids is None else env_ids
    for k in ("current_air_time", "last_air_time", "current_contact_time", "last_contact_time"):
      self._air[k][e] = 0.0
    self._air["last_time"][e] = self._data.time[e]

  def reset_masked(self, mask):
    if self._air is None:
      return
    m = mask.unsqueeze(1)
    for k in ("current_air_time", "last_air_time", "current_contact_time", "last_contact_time"):
      self._air[k].masked_fill_(m, 0.0)
    self._air["last_time"].copy_(torch.where(mask, self._data.time, self._air["last_time"]))

  def update(self, dt):
    if self._air is None or "found" not in self._fields:
      return
    if self.engine_owned:
      raise RuntimeError(f"ContactSensor '{self.name}': the engine updates the air times of this "
                         "sensor (a fused env step owns them); release the fused step first")
    s = self._air
    found = self._extract().found
    now = self._data.time
    el = (now - s["last_time"]).unsqueeze(-1)
    contact = found > 0
    first_contact = (s["current_air_time"] > 0) & contact
    first_detached = (s["current_contact_time"] > 0) & ~contact
    s["last_air_time"].copy_(torch.where(first_contact, s["current_air_time"] + el, s["last_air_time"]))
    s["current_air_time"].copy_(torch.where(~contact, s["current_air_time"] + el, torch.zeros_like(el)))
    s["last_contact_time"].copy_(torch.where(first_detached, s["current_contact_time"] + el,
                                             s["last_contact_time"]))
    s["current_contact_time"].copy_(torch.where(contact, s["current_contact_time"] + el,
                                                torch.zeros_like(el)))
    s["last_time"].copy_(now)

  def compute_first_contact(self, dt: float, abs_tol: float = 1.0e-8) -> torch.Tensor:
    c = self._air["current_contact_time"]
    return (c > 0.0) & (c < dt + abs_tol)

  def compute_first_air(self, dt: float, abs_tol: float = 1.0e-8) -> torch.Tensor:
    a = self._air["current_air_time"]
    return (a > 0.0) & (a < dt + abs_tol)


class Terrain:
  """The env-origin state of a generated terrain (`terrains/terrain_importer.py:186-244`):
  sub-terrain spawn origins [rows, cols, 3], each env's level (row) and type (column), and
  the level moves of the terrain curriculum.  `update_env_origins_masked` is the
  sync-free form (reset mask, no host sync) of `update_env_origins`."""

  def __init__(self, terrain_origins, size, num_envs: int, device: str, max_init_terrain_level=None):
    from .terrains import curriculum_env_origins
    o, lv, ty = curriculum_env_origins(terrain_origins, num_envs, max_init_terrain_level)
    self.terrain_origins = torch.as_tensor(np.asarray(terrain_origins), dtype=torch.float32, device=device)
    self.env_origins = o.to(device)
    self.terrain_levels, self.terrain_types = lv.to(device), ty.to(device)
    self.max_terrain_level = int(self.terrain_origins.shape[0])
    self.size = size
    self.mean_level = torch.zeros((), device=device)

  def update_env_origins(self, env_ids, move_up, move_down):
    lv = self.terrain_levels[env_ids] + 1 * move_up - 1 * move_down
    lv = torch.where(lv >= self.max_terrain_level,
                     torch.randint_like(lv, self.max_terrain_level), torch.clip(lv, 0))
    self.terrain_levels[env_ids] = lv
    self.env_origins[env_ids] = self.terrain_origins[self.terrain_levels[env_ids],
                                                     self.terrain_types[env_ids]]

  def update_env_origins_masked(self, mask, move_up, move_down):
    lv = self.terrain_levels + move_up.long() - move_down.long()
    lv = torch.where(lv >= self.max_terrain_level,
                     torch.randint_like(lv, self.max_terrain_level), lv.clamp(min=0))
    self.terrain_levels.copy_(torch.where(mask, lv, self.terrain_levels))
    self.env_origins.copy_(torch.where(mask.unsqueeze(1),
                                       self.terrain_origins[self.terrain_levels, self.terrain_types],
                                       self.env_origins))
    self.mean_level.copy_(self.terrain_levels.float().mean())

  def update_env_origins_native(self, mask, xpos, root_body: int, command, episode_length_s: float):
    """The terrain-level curriculum of the resetting envs as one HIP kernel
    (`mjx_terrain_levels`: the rule of `terrain_levels_vel` + `update_env_origins`, and the
    mean level), in place of ~13 torch launches.  Its wrap-around draw is a counter hash,
    not torch's generator."""
    import ctypes
    from ._lib import lib
    L = lib()
    if not hasattr(self, "_counter"):
      self._counter = torch.zeros(1, dtype=torch.int64, device=self.env_origins.device)
      self._seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    for t in (mask, xpos, command, self.terrain_levels, self.terrain_types, self.terrain_origins,
              self.env_origins):
      assert t.is_contiguous()
    vp = ctypes.c_void_p
    stream = vp(torch.cuda.current_stream(self.env_origins.device).cuda_stream)
    n, nb = int(xpos.shape[0]), int(xpos.shape[1])
    rc = L.mjx_terrain_levels(n, vp(mask.data_ptr()), vp(xpos.data_ptr()), nb, int(root_body),
                              vp(command.data_ptr()), float(self.size[0] / 2), float(episode_length_s),
                              vp(self.terrain_types.data_ptr()), vp(self.terrain_levels.data_ptr()),
                              vp(self.terrain_origins.data_ptr()), int(self.terrain_origins.shape[0]),
                              int(self.terrain_origins.shape[1]), vp(self.env_origins.data_ptr()),
                              ctypes.c_uint64(self._seed), vp(self._counter.data_ptr()),
                              vp(self.mean_level.data_ptr()), stream)
    if rc != 0:
      from ._lib import MjxError
      raise MjxError(L.mjx_task_last_error().decode())

  def randomize_env_origins_masked(self, mask) -> None:
    """randomize_env_origins over a reset mask (sync-free, graph-capturable): every env
    draws, the unmasked keep their level, type and origin."""
    rows, cols = self.terrain_origins.shape[:2]
    n = self.env_origins.shape[0]
    dev = self.env_origins.device
    lv = torch.randint(0, rows, (n,), device=dev)
    ty = torch.randint(0, cols, (n,), device=dev)
    self.terrain_levels.copy_(torch.where(mask, lv, self.terrain_levels))
    self.terrain_types.copy_(torch.where(mask, ty, self.terrain_types))
    self.env_origins.copy_(torch.where(mask.unsqueeze(1),
                                       self.terrain_origins[self.terrain_levels, self.terrain_types],
                                       self.env_origins))

  def randomize_env_origins(self, env_ids) -> None:
    """`terrain_importer.py:203-222` (play mode)."""
    rows, cols = self.terrain_origins.shape[:2]
    n = len(env_ids)
    self.terrain_levels[env_ids] = torch.randint(0, rows, (n,), device=self.env_origins.device)
    self.terrain_types[env_ids] = torch.randint(0, cols, (n,), device=self.env_origins.device)
    self.env_origins[env_ids] = self.terrain_origins[self.terrain_levels[env_ids],
                                                     self.terrain_types[env_ids]]


@dataclass(kw_only=True)
class SceneCfg:
  """`scene/scene.py:18-26`."""
  num_envs: int = 1
  env_spacing: float = 2.0
  terrain: object | None = None        # terrains.TerrainImporterCfg
  entities: dict = field(default_factory=dict)   # name -> entity.EntityCfg
  sensors: tuple = field(default_factory=tuple)  # sensor.ContactSensorCfg, ...
  extent: float | None = None
  spec_fn: object | None = None


class Scene:
  """The scene of an env (`scene/scene.py:29-198`): built from a `SceneCfg` at env
  construction -- terrain, each entity's spec attached under `<name>/`, the contact sensors
  expanded over the entities, the merged keyframe -- and compiled by `compile()` into the
  flat model the engine loads.  `initialize` then binds the runtime views (entities,
  sensors, env origins) to the simulation's device fields."""

  def __init__(self, scene_cfg: SceneCfg, device: str):
    from .entity import EntityBuild
    if scene_cfg.spec_fn is not None:
      raise NotImplementedError("SceneCfg.spec_fn: scene-level MjSpec edits (edit the entity "
                                "specs through EntityCfg.spec_fn instead)")
    self._cfg = scene_cfg
    self.num_envs = int(scene_cfg.num_envs)
    self.device = device
    self._builds = {name: EntityBuild(name, ecfg) for name, ecfg in scene_cfg.entities.items()}
    self._terrain_geoms, self._terrain_origins, self._terrain_size = None, None, None
    t = scene_cfg.terrain
    self._terrain_kind = "none"
    if t is not None:
      t.num_envs = self.num_envs
      t.env_spacing = scene_cfg.env_spacing
      if t.terrain_type == "plane":
        self._terrain_kind = "plane"
      elif t.terrain_type == "generator":
        from .terrains import TerrainGenerator
        if t.terrain_generator is None:
          raise ValueError("terrain_type 'generator' needs a terrain_generator cfg")
        self._terrain_kind = "generator"
        geoms, origins = TerrainGenerator(t.terrain_generator).generate()
        self._terrain_geoms, self._terrain_origins = geoms, origins
        self._terrain_size = tuple(float(v) for v in t.terrain_generator.size)
      else:
        raise ValueError(f"unknown terrain_type {t.terrain_type!r}")
    from .sensor import BuiltinSensorCfg
    xml_sensors = {f"{n}/{a.get('name', '')}" for n, b in self._builds.items()
                   for _, a in b.spec._xml.sensors}
    self._sensor_cfgs = {}
    self._contact_specs = []
    for sc in scene_cfg.sensors:
      if not hasattr(sc, "expand"):
        raise NotImplementedError(f"sensor cfg {type(sc).__name__}")
      if isinstance(sc, BuiltinSensorCfg) and sc.name in xml_sensors | set(self._sensor_cfgs):
        if sc.obj is not None and sc.obj.entity is not None:
          raise ValueError(f"Sensor '{sc.name}' is defined in both entity XML and scene config. "
                           "Remove the sensor definition from the entity XML file, or remove the "
                           "BuiltinSensorCfg from scene.sensors.")
        raise ValueError(f"Sensor '{sc.name}' already exists in the scene. Rename this sensor "
                         "to avoid conflicts.")
      self._contact_specs.append(sc.expand(self._builds))
      if not isinstance(sc, BuiltinSensorCfg):
        self._sensor_cfgs[sc.name] = sc
    self._model = None

  @classmethod
  def for_model(cls, mj_model, num_envs: int, device: str, entities: dict | None = None):
    """Runtime views over an already compiled model, without a SceneCfg: `entities` maps
    entity names to their soft joint-limit factor ({"robot": 0.9} by default).  The motion
    tools (`tracking.synthesize_motion`, `motion_csv.csv_to_npz`) record frames through
    the engine this way, as the reference's `csv_to_npz` builds a bare scene."""
    from types import SimpleNamespace
    from .entity import EntityArticulationInfoCfg, EntityCfg
    self = cls.__new__(cls)
    self._cfg = SceneCfg(num_envs=num_envs)
    self.num_envs, self.device = int(num_envs), device
    self._builds = {n: SimpleNamespace(cfg=EntityCfg(articulation=EntityArticulationInfoCfg(
        soft_joint_pos_limit_factor=f))) for n, f in (entities or {"robot": 0.9}).items()}
    self._terrain_geoms = self._terrain_origins = self._terrain_size = None
    self._terrain_kind = "none"
    self._sensor_cfgs, self._contact_specs = {}, []
    self._model = mj_model
    return self

  def compile(self):
    """`MjSpec.compile()` of the assembled scene (scene/scene.py:47-48)."""
    from .compiler.model import compile_scene
    ents = [b.entity_spec() for b in self._builds.values()]
    m = compile_scene(ents, terrain=self._terrain_kind, terrain_geoms=self._terrain_geoms,
                      contact_sensors=self._contact_specs)
    if self._terrain_origins is not None:
      m.arrays["terrain_origins"] = np.asarray(self._terrain_origins, np.float64)
      m.arrays["terrain_size"] = np.asarray(self._terrain_size, np.float64)
    self._model = m
    return m

  @property
  def cfg(self) -> SceneCfg:
    return self._cfg

  @property
  def env_spacing(self) -> float:
    return self._cfg.env_spacing

  def _bind(self, mj_model) -> None:
    """Runtime entities and sensors over the compiled model's name tables."""
    self._m = mj_model
    self._entities = {}
    for name, b in self._builds.items():
      art = b.cfg.articulation
      init = b.cfg.init_state
      self._entities[name] = Entity(
        name, mj_model, soft_joint_pos_limit_factor=art.soft_joint_pos_limit_factor if art else 1.0,
        init_lin_vel=init.lin_vel, init_ang_vel=init.ang_vel)
    self._sensors = {}
    names = mj_model.names["sensor"]
    adr, dim = mj_model.sensor_adr, mj_model.sensor_dim
    for i, n in enumerate(names):
      if mj_model.sensor_type[i] != 4:  # builtin
        self._sensors[n] = BuiltinSensor(n, int(adr[i]), int(dim[i]))
    for cname, sc in self._sensor_cfgs.items():
      slots = []
      for i, n in enumerate(names):
        if mj_model.sensor_type[i] == 4 and n.startswith(cname + "_"):
          prim, fld = n[len(cname) + 1:].rsplit("_", 1)
          slots.append((prim, fld, int(adr[i]), int(dim[i])))
      self._sensors[cname] = ContactSensor(cname, slots, sc.fields, sc.num_slots, sc.track_air_time)
    self.terrain = None
    t = self._cfg.terrain
    if "terrain_origins" in mj_model.arrays:
      # generator terrain: curriculum origins over the sub-terrain spawn points
      # (terrain_importer.py:224-244), drawn from torch's global RNG like the reference
      size = tuple(float(v) for v in mj_model.arrays.get("terrain_size", (8.0, 8.0)))
      self.terrain = Terrain(mj_model.arrays["terrain_origins"], size, self.num_envs, self.device,
                             t.max_init_terrain_level if t is not None else None)
      self.env_origins = self.terrain.env_origins
      self.terrain_levels, self.terrain_types = self.terrain.terrain_levels, self.terrain.terrain_types
      return
    if t is None:
      # no terrain: every env at the origin (scene/scene.py:128-130)
      self.env_origins = torch.zeros(self.num_envs, 3, device=self.device)
      return
    # plane: env origins on a grid (terrain_importer.py:246-261)
    num_envs, spacing = self.num_envs, float(self._cfg.env_spacing)
    rows = int(np.ceil(num_envs / int(np.sqrt(num_envs))))
    cols = int(np.ceil(num_envs / rows))
    ii, jj = torch.meshgrid(torch.arange(rows, device=self.device),
                            torch.arange(cols, device=self.device), indexing="ij")
    o = torch.zeros(num_envs, 3, device=self.device)
    o[:, 0] = -(ii.flatten()[:num_envs] - (rows - 1) / 2) * spacing
    o[:, 1] = (jj.flatten()[:num_envs] - (cols - 1) / 2) * spacing
    self.env_origins = o

  def __getitem__(self, key):
    if key == "terrain":
      if self.terrain is None:
        raise KeyError("No terrain configured in this scene.")
      return self.terrain
    if key in self._sensors:
      return self._sensors[key]
    if key in self._entities:
      return self._entities[key]
    available = list(self._entities) + list(self._sensors)
    raise KeyError(f"Scene element '{key}' not found. Available: {available}")

  @property
  def entities(self):
    return self._entities

  @property
  def sensors(self):
    return self._sensors

  def initialize(self, mj_model, model, data):
    self._bind(mj_model)
    for e in self._entities.values():
      e.initialize(mj_model, model, data, self.device)
    for s in self._sensors.values():
      if isinstance(s, ContactSensor):
        s.initialize(data, self.device)
      else:
        s.initialize(data)

  def reset(self, env_ids=None):
    for e in self._entities.values():
      e.reset(env_ids)
    for s in self._sensors.values():
      s.reset(env_ids)

  def reset_masked(self, mask):
    for e in self._entities.values():
      e.reset_masked(mask)
    for s in self._sensors.values():
      s.reset_masked(mask)

  def update(self, dt: float):
    for e in self._entities.values():
      e.update(dt)
    for s in self._sensors.values():
      s.update(dt)

  def write_data_to_sim(self):
    for e in self._entities.values():
      e.write_data_to_sim()
