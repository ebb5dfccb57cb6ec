"""--env-backend gym: real gym envs behind the vectorised-env surface.

gym is not installed in this image, so these tests install an in-test env with gym's
``reset()/step()`` API through ``register_env`` (the same hook ``gym.make`` is the default of);
parity with the reference's MuJoCo curves is unpinned.  The surface matched is
``main.py:45`` / ``train.py:48`` (``gym.make(env_name)``; ``observation_space.shape[0]``,
``action_space.shape[0]``) and the auto-reset of ``train.py:98-105``.
"""
import math

import numpy as np
import pytest
import torch

from pytorch_dppo_amd.config import dppo_preset
from pytorch_dppo_amd.envs import GymVecEnv, make_vec_env, register_env


class _Box:
    def __init__(self, n):
        self.shape = (n,)


class _Spec:
    max_episode_steps = 12


class FakeGymEnv:
    """old-gym-API env: s' = 0.9 s + 0.1 tanh(a) (padded), r = -|a - tanh(s[:A])|^2, terminal
    when |s0| > 2; TimeLimit 12 steps via ``spec.max_episode_steps``."""
    O, A = 5, 2

    def __init__(self):
        self.observation_space = _Box(self.O)
        self.action_space = _Box(self.A)
        self.spec = _Spec()
        self.rs = np.random.RandomState(0)
        self.s = np.zeros(self.O)

    def seed(self, s):
        self.rs = np.random.RandomState(s)

    def reset(self):
        self.s = self.rs.randn(self.O) * 0.5
        return self.s.astype(np.float32)

    def step(self, a):
        a = np.asarray(a, dtype=np.float64)
        r = -float(((a - np.tanh(self.s[:self.A])) ** 2).sum())
        drive = np.zeros(self.O)
        drive[:self.A] = np.tanh(a)
        self.s = 0.9 * self.s + 0.1 * drive + 0.05 * self.rs.randn(self.O)
        return self.s.astype(np.float32), r, bool(abs(self.s[0]) > 2.0), {}


register_env("FakeGym-v0", FakeGymEnv)


def test_gym_vec_env_surface_and_time_limit():
    env = make_vec_env(None, 3, seed=4, backend="gym", name="FakeGym-v0")
    assert isinstance(env, GymVecEnv) and env.host_stepped
    assert (env.E, env.O, env.A, env.limit) == (3, 5, 2, 12)
    obs = env.reset()
    assert obs.shape == (3, 5) and torch.equal(env.observe(), obs)
    total_done = 0
    for t in range(12):
        obs, r, done, info = env.step(torch.zeros(3, 2))
        total_done += int(done.sum())
        assert obs.shape == (3, 5) and r.shape == (3,)
    assert total_done >= 3 and int(info["ep_count"]) >= 0     # every env hit the 12-step limit
    assert env.t == 12 and torch.equal(env.env_idx, torch.arange(3))
    with pytest.raises(RuntimeError):
        env.kernel_params()
    with pytest.raises(ValueError):
        make_vec_env(None, 1, backend="mujoco", name="FakeGym-v0")


def test_missing_gym_raises_clearly():
    with pytest.raises(RuntimeError, match="gym"):
        GymVecEnv("Humanoid-v2-not-registered", 1)


def test_params_env_backend_flag():
    from pytorch_dppo_amd.config import params_from_args
    p = params_from_args(["--env-backend", "gym", "--env-name", "FakeGym-v0"])
    assert p.env_backend == "gym" and p.env_name == "FakeGym-v0"
    with pytest.raises(ValueError):
        dppo_preset(env_backend="mujoco")


def test_dppo_worker_trains_on_gym_backend_cpu():
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    p = dppo_preset(device="cpu", env_backend="gym", env_name="FakeGym-v0", num_envs=4, exploration_size=64,
                    batch_size=64, num_epoch=3, seed=2)
    w = DPPOWorker(p, DistContext(device=torch.device("cpu")))
    assert (w.spec.obs_dim, w.spec.act_dim) == (5, 2)
    m0 = w.iteration_step()
    m1 = w.iteration_step()
    assert math.isfinite(m1["loss"]) and m1["env_steps"] == 2 * 64
    assert w.env.t == 32
    assert m0["iteration"] == 1 and m1["updates"] == 6


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", ["bf16x3", "bf16"])
def test_hip_engine_host_env_path_matches_torch_engine(dtype):
    """GPU engine with a host-stepped gym env: the rollout runs the host path (env on the host,
    policy as device tensor ops, same keyed noise) and equals the torch engine's; then a full
    worker iteration runs its update on the HIP kernels."""
    from pytorch_dppo_amd.models.actor_critic import ActorCritic
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.engine_hip import HipEngine
    from pytorch_dppo_amd.runtime.engine_torch import TorchEngine
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    from pytorch_dppo_amd.utils.obs_stats import RunningObsStats
    dev = torch.device("cuda", 0)
    p = dppo_preset(device="gpu", env_backend="gym", env_name="FakeGym-v0", num_envs=16, exploration_size=16 * 8,
                    batch_size=16 * 8, num_epoch=2, dtype=dtype, seed=3)
    engines = []
    for cls in (HipEngine, TorchEngine):
        torch.manual_seed(0)
        model = ActorCritic(5, 2).to(dev)
        env = make_vec_env(None, p.num_envs, seed=p.seed, backend="gym", name="FakeGym-v0")
        st = RunningObsStats(5, dev)
        eng = cls(p, model, env, st, dev, 0)
        st.observes(eng.current_obs() if cls is HipEngine else eng.obs)
        eng.rollout()
        engines.append(eng)
    h, t = engines
    assert h.host_env
    T, E = h.T, h.E
    assert torch.allclose(h.actions.view(T, E, -1), t.actions, atol=1e-6)
    assert torch.allclose(h.logp.view(T, E), t.logp, atol=1e-6)
    assert torch.equal(h.dones.view(T, E), t.dones)
    tol = 1e-2 if dtype == "bf16" else 1e-4
    assert torch.allclose(h.decode(h.x_buf).view(T + 1, E, -1)[..., :5], t.x, atol=tol)
    w = DPPOWorker(p, DistContext(device=dev))
    m = w.iteration_step()
    assert math.isfinite(m["loss"]) and m["updates"] == 2


@pytest.mark.gpu
def test_hip_engine_host_env_fp8_refreshes_forward_image():
    """fp8 + host env: Adam rewrites only the bf16 image, so the rollout must refresh the e4m3
    forward image (and its scales) before the host path too — values() / GAE then use the current
    weights."""
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    dev = torch.device("cuda", 0)
    p = dppo_preset(device="gpu", env_backend="gym", env_name="FakeGym-v0", num_envs=16, exploration_size=16 * 8,
                    batch_size=16 * 8, num_epoch=2, dtype="fp8", seed=3)
    w = DPPOWorker(p, DistContext(device=dev))
    w.iteration_step()
    eng = w.engine
    eng.rollout()
    img, q = eng.wimg_fwd.clone(), eng.qscale.clone()
    eng.refresh_fwd_image()
    assert torch.equal(img, eng.wimg_fwd) and torch.equal(q, eng.qscale)


@pytest.mark.gpu
def test_hip_engine_host_env_resume_refreshes_observation():
    """after load_env_state the next host rollout acts on the restored envs' observation"""
    from pytorch_dppo_amd.models.actor_critic import ActorCritic
    from pytorch_dppo_amd.runtime.engine_hip import HipEngine
    from pytorch_dppo_amd.utils.obs_stats import RunningObsStats
    dev = torch.device("cuda", 0)
    p = dppo_preset(device="gpu", env_backend="gym", env_name="FakeGym-v0", num_envs=16, exploration_size=16 * 4,
                    batch_size=16 * 4, num_epoch=1, dtype="bf16x3", seed=3)
    engs = []
    for _ in range(2):
        torch.manual_seed(0)
        env = make_vec_env(None, p.num_envs, seed=p.seed, backend="gym", name="FakeGym-v0")
        st = RunningObsStats(5, dev)
        eng = HipEngine(p, ActorCritic(5, 2).to(dev), env, st, dev, 0)
        st.observes(eng.current_obs())
        engs.append(eng)
    a, b = engs
    a.rollout()
    b.load_env_state(a.env_state())
    assert torch.equal(b.current_obs().cpu(), b.env.observe().float())
