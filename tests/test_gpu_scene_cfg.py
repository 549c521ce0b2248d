"""A `cfg.scene` edit reaches the engine: the G1 velocity task with a
contact sensor added, the foot geoms' friction and the torso's mass changed in its SceneCfg;
the env is built from the edited cfg (Scene(scene_cfg, device) -> compile -> Simulation),
and its first physics steps match the oracle stepping the same edited model."""

import numpy as np
import pytest
import torch

import oracle_lib as ol
from parity_util import expanded_fields, world_model
from test_gpu_rollout_parity import _OUT, _STATE, _check_step, _snap
from scene_edits import edited_g1_cfg
from test_gpu_config1 import _stats

pytestmark = pytest.mark.gpu


def test_edited_scene_generic_kernels_warn(gpu_device):
  """specialize="never": the generic kernels run, and the user is told so.  (First in this
  file: the next test loads the run-time specialisation, which any later sim of these dims
  in the process then matches.)"""
  from mjlab_amd.envs import ManagerBasedRlEnv
  from mjlab_amd.sim.sim import GenericKernelWarning, _generic_warned
  cfg = edited_g1_cfg(16)
  cfg.sim.specialize = "never"
  _generic_warned.clear()
  with pytest.warns(GenericKernelWarning, match="no specialised step kernels"):
    env = ManagerBasedRlEnv(cfg, device=gpu_device)
  assert env.sim.info()["spec"] == 0



def test_edited_scene_cfg_reaches_the_engine(gpu_device):
  from mjlab_amd.envs import ManagerBasedRlEnv
  from mjlab_amd.scenes import load_scene
  cfg = edited_g1_cfg(16)
  # the edit adds sensors, so no compiled specs.inc entry matches: the kernels specialised for
  # it at run time (mjlab_amd.jit; __graft_entry__.build() compiled them into the in-tree
  # cache, so no compile happens here)
  cfg.sim.specialize = "always"
  env = ManagerBasedRlEnv(cfg, device=gpu_device)
  info = env.sim.info()
  assert info["spec"] >= 1000 and info["spec_max"] >= 1000, info  # run-time specialisations
  env.reset()
  sim = env.sim
  base = load_scene("g1_velocity")
  m = sim.mj_model
  torso = m.names["body"].index("robot/torso_link")
  assert float(sim.model.body_mass[0, torso]) == pytest.approx(base.body_mass[torso] + 2.5, rel=1e-6)
  feet = [i for i, n in enumerate(m.names["geom"]) if "_foot" in n and n.endswith("_collision")]
  assert len(feet) == 14
  assert torch.all(sim.model.geom_friction[0, feet, 0] == torch.tensor(0.9))
  assert env.scene["hands"].data.found.shape == (16, 2)
  assert env.scene["hands"].data.force.shape == (16, 2, 3)
  assert m.nsensordata == base.nsensordata + 8
  # the first substeps of the edited model, every world, against the oracle on the same model
  rng = np.random.default_rng(0)
  nact = env.action_manager.total_action_dim
  sel = np.arange(16)
  fields = expanded_fields(sim)
  models = {w: world_model(sim, w, fields) for w in sel}
  stats = _stats()
  for k in range(3):
    a = torch.as_tensor(rng.uniform(-1, 1, (16, nact)), dtype=torch.float32, device=gpu_device)
    env.action_manager.process_action(a)
    env.action_manager.apply_action()
    env.scene.write_data_to_sim()
    torch.cuda.synchronize()
    st0 = _snap(sim, sel, _STATE)
    sim.step()
    torch.cuda.synchronize()
    st1, out = _snap(sim, sel, _STATE), _snap(sim, sel, _OUT)
    for i, w in enumerate(sel):
      ref = ol.forward(models[w], st0["qpos"][i], st0["qvel"][i], st0["qacc_warmstart"][i],
                       st0["ctrl"][i], float(st0["time"][i].reshape(-1)[0]), step=True,
                       nconmax=sim.nconmax, njmax=sim.njmax)
      _check_step(models[w], ref, st0, st1, out, i, stats, f"edited scene world {w} substep {k}", sim)
  assert stats["checked"] >= 0.9 * 3 * 16
