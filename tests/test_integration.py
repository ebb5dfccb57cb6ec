"""Integration: CLI entrypoints, the evaluator process, and that training actually learns."""
import os
import subprocess
import sys

import pytest
import torch

from pytorch_dppo_amd.config import dppo_preset, ppo_preset
from pytorch_dppo_amd.parallel.dist import DistContext

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=240):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    return subprocess.run([sys.executable] + args, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)


@pytest.mark.slow
def test_train_py_ppo_preset_cli():
    r = _run(["train.py", "--preset", "ppo", "--env-name", "Pendulum-v0", "--num-envs", "4", "--exploration-size",
              "64", "--batch-size", "32", "--max-iters", "2", "--hidden", "16,16"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "iter 2" in r.stdout


@pytest.mark.slow
def test_main_py_shim_runs_dppo_with_two_workers():
    r = _run(["main.py", "--env-name", "InvertedPendulum-v1", "--num-processes", "2", "--num-envs", "4",
              "--exploration-size", "64", "--batch-size", "64", "--max-iters", "2", "--hidden", "16,16", "--num-epoch", "2"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert "iter 2" in r.stdout


@pytest.mark.slow
def test_evaluator_process_runs_episodes_on_snapshots(capfd):
    from pytorch_dppo_amd.models.actor_critic import ActorCritic
    from pytorch_dppo_amd.runtime.evaluator import EvaluatorHandle
    from pytorch_dppo_amd.utils.obs_stats import RunningObsStats
    p = dppo_preset(env_name="Pendulum-v0", hidden=(16, 16), eval_every=1)
    ev = EvaluatorHandle(p, results=True)
    try:
        m = ActorCritic(3, 1, (16, 16))
        st = RunningObsStats(3)
        st.observes(torch.randn(10, 3))
        assert ev.push(m.state_dict(), st.state_dict(), 7)
        res = ev.out_q.get(timeout=120)
        assert res["iteration"] == 7 and res["length"] == 200   # Pendulum-v0 TimeLimit
        assert res["return"] < 0
    finally:
        ev.close()


def test_dppo_learns_synthetic_task():
    """A few CPU iterations must raise the per-step reward of the learnable synthetic task."""
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    torch.set_num_threads(2)
    p = dppo_preset(env_name="Synthetic-6x2", num_envs=32, exploration_size=32 * 32, batch_size=256, num_epoch=4,
                    hidden=(32, 32), lr=3e-3, reward_clip=0.0)
    w = DPPOWorker(p, DistContext())
    rewards = []
    for _ in range(15):
        w.iteration_step()
        rewards.append(float(w.engine.rewards.mean()))
    assert rewards[-1] > rewards[0] + 0.05, rewards


def test_ppo_single_process_preset_learns_pendulum_direction():
    """ppo.py semantics (1 minibatch of 64 per epoch, grad clip 0.5): runs and stays finite."""
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    p = ppo_preset(env_name="Pendulum-v0", num_envs=8, exploration_size=256, hidden=(32, 32))
    w = DPPOWorker(p, DistContext())
    for _ in range(3):
        m = w.iteration_step()
    assert m["updates"] == 30 and torch.isfinite(w.model.flat.data).all()
    assert m["grad_norm"] > 0
