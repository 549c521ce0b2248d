"""The learner on the MI355X env step: PPO iterations on the graph-captured, fused G1
velocity env (mjlab_amd/rl, scripts/train.py flow): finite losses, the observation
normalisers see the rollouts, parameters move, and a checkpoint round-trips."""

import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_ppo_iterations_on_the_env(gpu_device, tmp_path):
  from mjlab_amd.envs import make_env
  from mjlab_amd.rl import OnPolicyRunner, RslRlVecEnvWrapper, load_rl_cfg
  torch.manual_seed(0)
  cfg = load_rl_cfg("Mjlab-Velocity-Flat-Unitree-G1")
  env = make_env("Mjlab-Velocity-Flat-Unitree-G1", num_envs=512, device=gpu_device, seed=1)
  vec = RslRlVecEnvWrapper(env)
  env.enable_graph(capture=True)
  assert env._fused is not None
  runner = OnPolicyRunner(vec, cfg, log_dir=str(tmp_path), device=gpu_device)
  before = [p.detach().clone() for p in runner.alg.policy.parameters()]
  hist = runner.learn(3, init_at_random_ep_len=True)
  assert len(hist) == 3
  for h in hist:
    assert all(math.isfinite(h[k]) for k in ("value_function", "surrogate", "entropy", "fps"))
  assert int(runner.alg.policy.actor_obs_normalizer.count) == 3 * 24 * 512
  moved = sum(float((a - b).abs().max()) for a, b in zip(before, runner.alg.policy.parameters()))
  assert moved > 0
  # the graph-replayed rollout evaluation equals the eager one (values, means, std)
  obs = vec.get_observations()
  with torch.inference_mode():
    graphed = [t.clone() for t in runner.alg._act_graphed(obs)]
    eager = runner.alg._act_core(obs, runner.alg._geps)  # same standard normals
    for i in range(5):
      torch.testing.assert_close(graphed[i], eager[i], rtol=1e-5, atol=1e-5)
  ckpt = tmp_path / "model_3.pt"
  assert ckpt.exists()
  runner2 = OnPolicyRunner(vec, cfg, device=gpu_device)
  runner2.load(str(ckpt))
  assert runner2.current_learning_iteration == 3
  obs = vec.get_observations()
  a1 = runner.get_inference_policy()(obs)
  a2 = runner2.get_inference_policy()(obs)
  torch.testing.assert_close(a1, a2)
  # graphs recorded during the rollout (inside inference mode) leave later captures made
  # outside it usable (the CUDA generator's graph state is not an inference tensor)
  x = torch.zeros(8, device=gpu_device)
  g = torch.cuda.CUDAGraph()
  with torch.cuda.graph(g):
    x.add_(1.0)
  g.replay()
  torch.cuda.synchronize()
  assert float(x.sum()) == 8.0
