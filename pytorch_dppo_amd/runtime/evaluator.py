"""Online evaluator — the reference ``test.py`` process (``test.py:24-65``).

Reference behaviour: reload the shared weights every env step (torn reads while the chief
writes, Q18), update the SHARED obs stats from the evaluator too (Q5), act stochastically
``mu + sqrt(sigma_sq)*eps``, print ``Time …, episode reward …, episode length …`` per
episode and sleep 10 s.

Here rank 0 hands the evaluator a consistent snapshot (reference-format state_dict + frozen
obs stats) every ``eval_every`` iterations through a bounded queue (dropped if the evaluator
is busy — the trainer never blocks on it).  The evaluator runs on the CPU in its own process,
keeps the print format, and never writes training state.
"""
from __future__ import annotations

import queue
import time
from typing import Dict, Optional

import torch

from ..envs import get_spec, host_spec, make_vec_env
from ..models.actor_critic import ActorCritic
from ..utils import rng
from ..utils.obs_stats import RunningObsStats


def run_episode(model: ActorCritic, stats: RunningObsStats, env, key_action: int,
                convention: str, max_steps: int = 100000, deterministic: bool = False):
    obs = env.reset()
    total, length = 0.0, 0
    dims = torch.arange(env.A, dtype=torch.int64)
    with torch.no_grad():
        while length < max_steps:
            x = stats.normalize(obs)
            mu, log_std, _ = model(x)
            if deterministic:
                a = mu
            else:
                sig = torch.exp(log_std if convention == "std" else 0.5 * log_std)
                eps = rng.gauss(key_action, env.env_idx[:, None], env.t, dims[None, :])
                a = mu + sig * eps
            obs, r, done, info = env.step(a)
            total += float(r[0])
            length += 1
            if bool(done[0]):
                break
    return total, length


def evaluator_main(params_dict: Dict, q, stop_event=None, out_q=None) -> None:
    from ..config import Params
    p = Params.from_dict(params_dict)
    torch.set_num_threads(1)
    if p.env_backend == "gym":   # test.py:28 gym.make
        env = make_vec_env(None, 1, seed=p.seed + 7777, rank=0, max_episode_length=p.max_episode_length,
                           backend="gym", name=p.env_name)
        spec = host_spec(p.env_name, env.O, env.A, env.limit)
    else:
        spec = get_spec(p.env_name)
        env = make_vec_env(spec, 1, seed=p.seed + 7777, rank=0, device="cpu",
                           max_episode_length=p.max_episode_length)
    model = ActorCritic(spec.obs_dim, spec.act_dim, p.hidden, p.value_mult)
    stats = RunningObsStats(spec.obs_dim)
    key = rng.base_key(p.seed, rng.STREAM_EVAL, 0)
    start = time.time()
    while True:
        if stop_event is not None and stop_event.is_set():
            break
        try:
            snap = q.get(timeout=0.5)
        except queue.Empty:
            continue
        if snap is None:
            break
        model.load_state_dict(snap["model"])
        stats.load_state_dict(snap["obs_stats"])
        for _ in range(max(1, p.eval_episodes)):
            ret, length = run_episode(model, stats, env, key, p.std_convention)
            # test.py:56-59 print format
            print("Time {}, episode reward {}, episode length {}".format(
                time.strftime("%Hh %Mm %Ss", time.gmtime(time.time() - start)), ret, length),
                flush=True)
            if out_q is not None:
                out_q.put({"iteration": snap.get("iteration", -1), "return": ret, "length": length})
            if p.eval_sleep > 0:
                time.sleep(p.eval_sleep)


class EvaluatorHandle:
    """rank-0 side: spawn the evaluator process and push snapshots without blocking."""

    def __init__(self, params, results: bool = False):
        import torch.multiprocessing as mp
        ctx = mp.get_context("spawn")
        self.q = ctx.Queue(maxsize=1)
        self.out_q = ctx.Queue() if results else None
        self.stop = ctx.Event()
        self.proc = ctx.Process(target=evaluator_main, args=(params.to_dict(), self.q, self.stop, self.out_q),
                                daemon=True)
        self.proc.start()

    def push(self, model_sd: Dict, stats_sd: Dict, iteration: int) -> bool:
        try:
            self.q.put_nowait({"model": model_sd, "obs_stats": stats_sd, "iteration": iteration})
            return True
        except queue.Full:
            return False

    def close(self, timeout: float = 10.0) -> None:
        try:
            self.q.put(None, timeout=timeout)
        except Exception:
            pass
        self.stop.set()
        self.proc.join(timeout)
        if self.proc.is_alive():
            self.proc.terminate()
