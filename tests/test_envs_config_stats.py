"""Envs, config presets/CLI and running obs statistics."""
import math

import pytest
import torch

from pytorch_dppo_amd.config import Params, dppo_preset, params_from_args, ppo_preset
from pytorch_dppo_amd.envs import get_spec, known_envs, make_vec_env
from pytorch_dppo_amd.envs.registry import KIND_PENDULUM
from pytorch_dppo_amd.utils import rng
from pytorch_dppo_amd.utils.obs_stats import RunningObsStats


# ---------------- config ----------------
def test_dppo_preset_is_reference_main_params():
    p = dppo_preset()
    assert (p.batch_size, p.lr, p.gamma, p.gae_param, p.clip, p.ent_coeff) == (1000, 3e-4, 0.99, 0.95, 0.2, 0.0)
    assert (p.num_epoch, p.num_steps, p.exploration_size, p.num_processes) == (10, 1000, 1000, 4)
    assert p.update_treshold == 3 and p.update_threshold == 3
    assert (p.max_episode_length, p.seed, p.env_name) == (10000, 1, "InvertedPendulum-v1")


def test_ppo_preset_is_reference_ppo_params():
    p = ppo_preset()
    assert (p.batch_size, p.lr, p.ent_coeff, p.num_steps, p.max_grad_norm) == (64, 7e-4, 0.01, 2048, 0.5)
    assert (p.time_horizon, p.env_name) == (1000000, "HalfCheetah-v1")


def test_cli_flags_mirror_field_names():
    p = params_from_args(["--preset", "ppo", "--gae-param", "0.9", "--hidden", "64,64", "--num-envs", "8",
                          "--update-treshold", "5", "--compat", "--dtype", "bf16"])
    assert p.gae_param == 0.9 and p.hidden == (64, 64) and p.num_envs == 8
    assert p.update_treshold == 5 and p.compat is True and p.dtype == "bf16"
    q = Params.from_dict(p.to_dict())
    assert q == p


def test_dppo_ref_loss_forces_variance_convention():
    assert Params(loss="dppo_ref").std_convention == "var"


def test_rollout_geometry():
    p = Params(exploration_size=1000, num_envs=64, batch_size=256)
    assert p.rollout_len == 16 and p.buffer_rows == 1024
    assert p.minibatch_rows() == 256 and p.num_minibatches() == 4


# ---------------- envs ----------------
def test_registry_dims():
    assert (get_spec("Humanoid-v2").obs_dim, get_spec("Humanoid-v2").act_dim) == (376, 17)
    assert (get_spec("HalfCheetah-v1").obs_dim, get_spec("HalfCheetah-v1").act_dim) == (17, 6)
    assert get_spec("Pendulum-v0").kind == KIND_PENDULUM
    for name in ("InvertedPendulum-v1", "Reacher-v1", "Hopper-v1", "Ant-v1", "Humanoid-v1",
                 "InvertedDoublePendulum-v1", "HalfCheetahBulletEnv-v0", "HopperBulletEnv-v0", "AntBulletEnv-v0"):
        assert name in known_envs()


def test_pendulum_dynamics_follow_gym_pendulum_v0():
    env = make_vec_env(get_spec("Pendulum-v0"), 4)
    env.reset()
    s0 = env.state.clone()
    a = torch.tensor([[0.5], [-3.0], [2.0], [0.0]])
    obs, r, done, _ = env.step(a)
    for i in range(4):
        th, thd = float(s0[i, 0]), float(s0[i, 1])
        u = max(-2.0, min(2.0, float(a[i, 0])))
        thn = ((th + math.pi) % (2 * math.pi)) - math.pi
        cost = thn ** 2 + 0.1 * thd ** 2 + 0.001 * u ** 2
        nthd = thd + (-3 * 10 / 2 * math.sin(th + math.pi) + 3.0 * u) * 0.05
        nth = th + nthd * 0.05
        nthd = max(-8.0, min(8.0, nthd))
        assert abs(float(r[i]) + cost) < 1e-4
        assert abs(float(obs[i, 0]) - math.cos(nth)) < 1e-4 and abs(float(obs[i, 2]) - nthd) < 1e-4


def test_pendulum_time_limit_200():
    env = make_vec_env(get_spec("Pendulum-v0"), 2)
    env.reset()
    dones = [bool(env.step(torch.zeros(2, 1))[2][0]) for _ in range(200)]
    assert dones[-1] and not any(dones[:-1])


def test_synthetic_env_deterministic_and_keyed_by_rank():
    spec = get_spec("Walker2d-v2")
    e1 = make_vec_env(spec, 8, seed=3, rank=0)
    e2 = make_vec_env(spec, 8, seed=3, rank=0)
    e3 = make_vec_env(spec, 8, seed=3, rank=1)
    for e in (e1, e2, e3):
        e.reset()
    a = torch.randn(8, 6)
    o1 = e1.step(a)[0]
    o2 = e2.step(a)[0]
    o3 = e3.step(a)[0]
    assert torch.equal(o1, o2) and not torch.equal(o1, o3)


def test_synthetic_reward_is_learnable_target():
    env = make_vec_env(get_spec("Synthetic-4x2"), 16)
    env.reset()
    s = env.state.clone()
    good = torch.tanh(s[:, :2])
    r_good = env._dynamics(good, 0)[1]
    r_bad = env._dynamics(-good - 0.5, 0)[1]
    assert torch.all(r_good > r_bad) and torch.allclose(r_good, torch.ones(16))


def test_rng_gauss_statistics():
    e = torch.arange(20000)
    z = rng.gauss(rng.base_key(1, rng.STREAM_ACTION, 0), e, 5, torch.zeros_like(e))
    assert abs(z.mean().item()) < 0.03 and abs(z.std().item() - 1) < 0.03
    assert rng.hash_py(0x12345678) == int(rng._hash(torch.tensor([0x12345678]))[0])


# ---------------- obs stats ----------------
def _welford_sequential(xs, floor=1e-2):
    n, mean, md = 0, torch.zeros(xs.shape[1], dtype=torch.float64), torch.zeros(xs.shape[1], dtype=torch.float64)
    for x in xs.double():
        n += 1
        last = mean.clone()
        mean = mean + (x - mean) / n
        md = md + (x - last) * (x - mean)
    return n, mean, md, torch.clamp(md / n, min=floor)


def test_batched_merge_equals_reference_sequential_welford():
    g = torch.Generator().manual_seed(0)
    xs = torch.randn(300, 5, generator=g) * torch.tensor([1.0, 10.0, 0.01, 3.0, 100.0]) + 50.0
    st = RunningObsStats(5)
    for chunk in xs.split([1, 7, 92, 200]):
        st.observes(chunk)
    n, mean, md, var = _welford_sequential(xs)
    assert st.n == n
    assert torch.allclose(st.mean, mean, rtol=1e-10, atol=1e-9)
    assert torch.allclose(st.mean_diff, md, rtol=1e-8)
    assert torch.allclose(st.var, var, rtol=1e-8)


def test_normalize_clamps_to_5():
    st = RunningObsStats(2)
    st.observes(torch.tensor([[0.0, 0.0], [0.0, 0.0]]))
    out = st.normalize(torch.tensor([[100.0, -100.0]]))
    assert torch.equal(out, torch.tensor([[5.0, -5.0]]))  # var floor 1e-2 -> std 0.1


def test_obs_stats_state_dict_uses_reference_names():
    st = RunningObsStats(3)
    st.observes(torch.randn(10, 3))
    sd = st.state_dict()
    assert set(sd) == {"n", "mean", "mean_diff", "var"}
    st2 = RunningObsStats(3)
    st2.load_state_dict(sd)
    assert torch.equal(st2.mean, st.mean) and st2.n == st.n


# ---------------- API parity utilities ----------------
def test_counter_and_traffic_light_over_store():
    import torch.distributed as dist
    from pytorch_dppo_amd.utils.sync import Counter, TrafficLight
    store = dist.HashStore()
    c, light = Counter(store), TrafficLight(store)
    assert c.get() == 0 and light.get() is False
    for _ in range(3):
        c.increment()
    assert c.get() == 3
    c.reset()
    assert c.get() == 0
    before = light.get()
    light.switch()
    assert light.get() != before


def test_replay_memory_reference_api():
    from pytorch_dppo_amd.utils.sync import ReplayMemory
    mem = ReplayMemory(5, seed=0)
    states = [torch.full((1, 2), float(i)) for i in range(7)]
    acts = [torch.full((1, 1), float(i)) for i in range(7)]
    mem.push([states, acts])
    assert len(mem) == 5                       # FIFO eviction kept the last 5
    s, a = mem.sample(5)
    assert s.shape == (5, 2) and a.shape == (5, 1)
    assert sorted(a.view(-1).tolist()) == [2.0, 3.0, 4.0, 5.0, 6.0]
    mem.clear()
    assert len(mem) == 0
