"""The reference's own hot-path tests (tests/test_gpu_reference_ports.py: contact sensor,
builtin sensor, nan_detection, encoder bias) run against the fp64 CPU oracle: the same test
bodies with the oracle-backed `Simulation` stand-in (tests/oracle_sim.py) behind the scene
and the env.  This pins the oracle to the answers the reference's tests hold (found on a
resting box, none in the air, air-time transitions, the accelerometer's support reading,
identical physics under encoder-bias compensation, ...) by a route independent of the engine,
which the GPU module then checks against the oracle."""

import inspect

import pytest
import torch

import oracle_sim
import test_gpu_reference_ports as ports

_SKIP = {"test_bridge_raises_on_setattr"}  # the engine's device bridge itself (GPU)
_CASES = []
for _name, _fn in inspect.getmembers(ports, inspect.isfunction):
  if not _name.startswith("test_") or _name in _SKIP:
    continue
  _params = inspect.signature(_fn).parameters
  if "reduce_mode" in _params:
    _CASES += [(_name, dict(reduce_mode=r)) for r in ("none", "mindist", "maxforce", "netforce")]
  else:
    _CASES.append((_name, {}))


class _CpuSim(oracle_sim.OracleSimulation):
  def __init__(self, num_envs, cfg, model, device):
    super().__init__(num_envs, cfg, model, "cpu")


@pytest.mark.parametrize("name,kw", _CASES, ids=[f"{n}{'-' + str(k['reduce_mode']) if k else ''}" for n, k in _CASES])
def test_reference_port_on_oracle(name, kw, monkeypatch):
  import mjlab_amd.envs as envs
  monkeypatch.setattr(ports, "Simulation", _CpuSim)
  monkeypatch.setattr(envs, "Simulation", _CpuSim)
  monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
  fn = getattr(ports, name)
  params = inspect.signature(fn).parameters
  if "mock_env_with_sim" in params:
    fn(ports.mock_env_with_sim.__wrapped__("cpu"))
  elif "device" in params:
    fn(device="cpu", **kw)
  else:
    fn(**kw)
