"""Multi-process tests on the gloo backend (SURVEY §4 'Distributed (fake backend)').

Every test spawns fresh python processes (spawn start method) rendezvousing on 127.0.0.1.
"""
import os
import time

import pytest
import torch
import torch.multiprocessing as mp

from pytorch_dppo_amd.config import Params, dppo_preset
from pytorch_dppo_amd.runtime.launcher import free_port

pytestmark = pytest.mark.slow


def _init(rank, world, port, timeout=60.0):
    from pytorch_dppo_amd.parallel.dist import init_distributed
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    return init_distributed("cpu", rank=rank, world_size=world, timeout_s=timeout)


def _worker_grad_sum(rank, world, port, out_dir):
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    ctx = _init(rank, world, port)
    p = dppo_preset(env_name="HalfCheetah-v2", num_envs=8, exploration_size=64, batch_size=64, num_epoch=2,
                    verify_sync_every=1, num_processes=world)
    w = DPPOWorker(p, ctx)
    eng = w.engine
    w.init_stats()
    ro = eng.rollout()
    w._merge_stats(ro["count"], ro["s1"], ro["s2"], ro["shift"])
    eng.values()
    eng.gae()
    eng.begin_update()
    eng.grad(None)
    local = eng.grad_flat.clone()
    ctx.allreduce_grads(eng.grad_flat)
    reduced = eng.grad_flat.clone()
    eng.apply()
    m = w.iteration_step()
    torch.save({"local": local, "reduced": reduced, "flat": w.model.flat.data.clone(),
                "stats_mean": w.stats.mean.clone(), "stats_n": w.stats.n, "in_sync": m["replicas_in_sync"]},
               os.path.join(out_dir, f"r{rank}.pt"))
    ctx.destroy()


def _spawn(fn, world, *args):
    port = free_port()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=fn, args=(r, world, port) + args) for r in range(world)]
    for p in procs:
        p.start()
    return procs


def _join(procs, timeout):
    t0 = time.time()
    for p in procs:
        p.join(max(1.0, timeout - (time.time() - t0)))
    for p in procs:
        if p.is_alive():
            p.terminate()
    return [p.exitcode for p in procs]


def test_grad_allreduce_is_sum_and_replicas_stay_identical(tmp_path):
    codes = _join(_spawn(_worker_grad_sum, 2, str(tmp_path)), 240)
    assert codes == [0, 0]
    r0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    assert not torch.equal(r0["local"], r1["local"])          # different data per rank
    assert torch.allclose(r0["reduced"], r0["local"] + r1["local"], atol=1e-6)   # R1 = sum (model.py:55)
    assert torch.equal(r0["reduced"], r1["reduced"])
    assert torch.equal(r0["flat"], r1["flat"])                 # replicated Adam: bit-identical
    assert r0["in_sync"] and r1["in_sync"]
    assert torch.equal(r0["stats_mean"], r1["stats_mean"]) and r0["stats_n"] == r1["stats_n"]


def _worker_obs_merge(rank, world, port, out_dir):
    from pytorch_dppo_amd.utils.obs_stats import RunningObsStats
    ctx = _init(rank, world, port)
    g = torch.Generator().manual_seed(100 + rank)
    st = RunningObsStats(4)
    for _ in range(3):
        x = torch.randn(50, 4, generator=g) * (rank + 1) + rank
        shift = st.shift().clone()
        c, s1, s2 = RunningObsStats.moments(x, shift)
        c, s1, s2 = ctx.allreduce_obs_moments(c, s1, s2)
        st.merge_moments(c, s1, s2, shift)
    torch.save({"mean": st.mean, "md": st.mean_diff, "n": st.n}, os.path.join(out_dir, f"s{rank}.pt"))
    ctx.destroy()


def test_obs_stats_merge_equals_single_process_on_concatenated_stream(tmp_path):
    from pytorch_dppo_amd.utils.obs_stats import RunningObsStats
    assert _join(_spawn(_worker_obs_merge, 3, str(tmp_path)), 120) == [0, 0, 0]
    ref = RunningObsStats(4)
    gens = [torch.Generator().manual_seed(100 + r) for r in range(3)]
    for _ in range(3):
        xs = [torch.randn(50, 4, generator=gens[r]) * (r + 1) + r for r in range(3)]
        ref.observes(torch.cat(xs))
    for r in range(3):
        s = torch.load(tmp_path / f"s{r}.pt", weights_only=True)
        assert s["n"] == ref.n == 450
        assert torch.allclose(s["mean"], ref.mean, atol=1e-10)
        assert torch.allclose(s["md"], ref.mean_diff, rtol=1e-9)


def _worker_moments_extra(rank, world, port, out_dir):
    ctx = _init(rank, world, port)
    g = torch.Generator().manual_seed(7 + rank)
    s1, s2 = torch.randn(5, generator=g, dtype=torch.float64), torch.rand(5, generator=g, dtype=torch.float64)
    ep = torch.tensor([10.0 * (rank + 1), float(rank + 2)], dtype=torch.float64)
    c, r1, r2 = ctx.allreduce_obs_moments(64.0, s1, s2, count_uniform=True, extra=ep)
    torch.save({"s1": s1, "s2": s2, "c": c, "r1": r1, "r2": r2, "ep": ep}, os.path.join(out_dir, f"m{rank}.pt"))
    ctx.destroy()


def test_episode_stats_ride_on_the_moment_allreduce(tmp_path):
    """R2 + R5 in ONE collective: the episode [return sum, count] appended to the moment
    all-reduce come back summed over ranks, in place, and the moments are unchanged by it."""
    assert _join(_spawn(_worker_moments_extra, 3, str(tmp_path)), 120) == [0, 0, 0]
    ms = [torch.load(tmp_path / f"m{r}.pt", weights_only=True) for r in range(3)]
    s1 = sum(m["s1"] for m in ms)
    s2 = sum(m["s2"] for m in ms)
    for m in ms:
        assert m["c"] == 64.0 * 3
        assert torch.allclose(m["r1"], s1) and torch.allclose(m["r2"], s2)
        assert torch.equal(m["ep"], torch.tensor([60.0, 9.0], dtype=torch.float64))


def _worker_fault(rank, world, port, out_dir):
    ctx = _init(rank, world, port, timeout=20.0)
    if rank == 1:
        os._exit(3)  # injected fault: a worker dies (reference Q21 would deadlock the chief)
    t0 = time.time()
    try:
        for _ in range(100):
            ctx.allreduce_grads(torch.ones(1000))
            time.sleep(0.05)
        msg = "no error"
    except Exception as e:  # noqa: BLE001
        msg = f"error after {time.time() - t0:.1f}s: {type(e).__name__}"
    with open(os.path.join(out_dir, "fault.txt"), "w") as f:
        f.write(msg)


def test_dead_rank_makes_survivor_fail_fast_instead_of_deadlock(tmp_path):
    t0 = time.time()
    codes = _join(_spawn(_worker_fault, 2, str(tmp_path)), 120)
    assert codes[1] == 3
    msg = (tmp_path / "fault.txt").read_text()
    assert msg.startswith("error"), msg
    assert time.time() - t0 < 110


def _worker_hang(rank, world, port, out_dir):
    """rank 1 hangs OUTSIDE any collective (stuck host code); rank 0 is busy in a long
    non-collective phase: only the heartbeat can notice (collective timeout is 600 s here)."""
    from pytorch_dppo_amd.utils.heartbeat import start_heartbeat
    ctx = _init(rank, world, port, timeout=600.0)
    hb = start_heartbeat(ctx, 0.2, 1.5)   # default action: report + os._exit(75)
    if rank == 1:
        hb._stop.set()                     # the beacon thread dies with the "hung" process
        time.sleep(60)
        os._exit(0)
    time.sleep(60)
    os._exit(0)


def test_heartbeat_detects_a_hung_rank_outside_collectives(tmp_path):
    t0 = time.time()
    procs = _spawn(_worker_hang, 2, str(tmp_path))
    procs[0].join(30)
    code0 = procs[0].exitcode
    for p in procs:
        if p.is_alive():
            p.terminate()
            p.join(5)
    assert code0 == 75, code0
    assert time.time() - t0 < 30


def test_launcher_two_workers_checkpoint_and_resume(tmp_path):
    from pytorch_dppo_amd.runtime.launcher import launch
    ck = str(tmp_path / "ck")
    p = dppo_preset(env_name="Pendulum-v0", num_processes=2, num_envs=4, exploration_size=64, batch_size=64,
                    num_epoch=2, hidden=(16, 16), max_iters=2, checkpoint_dir=ck, log_jsonl=str(tmp_path / "log.jsonl"),
                    heartbeat_s=0.5)
    launch(p)
    assert os.path.exists(os.path.join(ck, "model.pt"))
    assert os.path.exists(os.path.join(ck, "env_rank1.pt"))
    lines = open(tmp_path / "log.jsonl").read().strip().splitlines()
    assert len(lines) == 2
    st = torch.load(os.path.join(ck, "trainer_state.pt"), weights_only=True)
    assert st["iteration"] == 2 and st["updates"] == 4 and st["world_size"] == 2
    p2 = Params.from_dict({**p.to_dict(), "resume": ck, "max_iters": 3, "checkpoint_dir": str(tmp_path / "ck2"),
                           "log_jsonl": ""})
    launch(p2)
    st2 = torch.load(os.path.join(str(tmp_path / "ck2"), "trainer_state.pt"), weights_only=True)
    assert st2["iteration"] == 3 and st2["updates"] == 6


def test_resume_continues_bit_identically_single_process(tmp_path):
    from pytorch_dppo_amd.parallel.dist import DistContext
    from pytorch_dppo_amd.runtime.launcher import run_worker
    base = dict(env_name="HalfCheetah-v2", num_processes=1, num_envs=8, exploration_size=64, batch_size=32,
                num_epoch=2, hidden=(32, 32))
    w_full, _ = run_worker(dppo_preset(max_iters=3, **base), DistContext(), evaluator=False, quiet=True)
    ck = str(tmp_path / "ck")
    run_worker(dppo_preset(max_iters=2, checkpoint_dir=ck, **base), DistContext(), evaluator=False, quiet=True)
    w_res, _ = run_worker(dppo_preset(max_iters=3, resume=ck, **base), DistContext(), evaluator=False, quiet=True)
    assert w_res.iteration == 3
    assert torch.equal(w_full.model.flat.data, w_res.model.flat.data)


def _worker_overlap(rank, world, port, out_dir):
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    ctx = _init(rank, world, port)
    res = {}
    for ov in (False, True):
        p = dppo_preset(env_name="HalfCheetah-v2", num_envs=8, exploration_size=64, batch_size=64, num_epoch=2,
                        overlap_rollout=ov, num_processes=world, verify_sync_every=1)
        w = DPPOWorker(p, ctx)
        for _ in range(3):
            m = w.iteration_step()
        w.flush_pending()
        res[ov] = (w.model.flat.data.clone(), m["replicas_in_sync"], w.updates, w.engine.adam_step)
    torch.save(res, os.path.join(out_dir, f"o{rank}.pt"))
    ctx.destroy()


def test_overlap_rollout_defers_last_step_but_applies_every_update(tmp_path):
    assert _join(_spawn(_worker_overlap, 2, str(tmp_path)), 240) == [0, 0]
    r0 = torch.load(tmp_path / "o0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "o1.pt", weights_only=True)
    for ov in (False, True):
        assert r0[ov][1] and r1[ov][1]                       # replicas identical in both modes
        assert r0[ov][2] == r0[ov][3] == 6                    # every update applied exactly once
        assert torch.equal(r0[ov][0], r1[ov][0])
    # the lagged rollouts see different weights -> a (slightly) different trajectory
    assert not torch.equal(r0[False][0], r0[True][0])


# ---- the native communicator's watchdog and collective-safe creation (mocked extension) --------

class _FakeCommExt:
    """stands in for the HIP extension's comm_* entry points (csrc/comm.cpp)"""

    def __init__(self, status_seq=(0,), fail_id=False, fail_init_rank=None, rank=0):
        self.status_seq = list(status_seq)
        self.fail_id, self.fail_init_rank, self.rank = fail_id, fail_init_rank, rank
        self.aborted, self.polls = [], 0

    def comm_unique_id(self):
        if self.fail_id:
            raise RuntimeError("RCCL ncclGetUniqueId failed: test")
        return b"x" * 128

    def comm_init(self, tok, n, rank, timeout_s):
        if self.fail_init_rank == rank:
            raise RuntimeError("RCCL ncclCommInitRankConfig timed out: test")
        return 7

    def comm_status(self, h):
        self.polls += 1
        return self.status_seq[min(self.polls - 1, len(self.status_seq) - 1)]

    def comm_abort(self, h):
        self.aborted.append(h)


class _NeverEvent:
    def query(self):
        return False

    def synchronize(self):
        raise AssertionError("the watchdog must poll, not block")


def test_watchdog_aborts_on_async_error():
    """an asynchronous RCCL error seen while waiting on the device -> ncclCommAbort + CollectiveError"""
    from pytorch_dppo_amd.parallel.dist import CollectiveError, DistContext, NativeComm
    ext = _FakeCommExt(status_seq=[0, 0, 0, 5])
    ctx = DistContext(rank=0, world_size=2, timeout_s=60.0)
    ctx.native = NativeComm(ext, 7, 2)
    t0 = time.time()
    with pytest.raises(CollectiveError, match="state 5"):
        ctx.wait_event(_NeverEvent())
    assert ext.aborted == [7] and time.time() - t0 < 10


def test_watchdog_aborts_after_timeout():
    """no completion within dist_timeout_s (a peer that died silently) -> abort + CollectiveError"""
    from pytorch_dppo_amd.parallel.dist import CollectiveError, DistContext, NativeComm
    ext, ext_side = _FakeCommExt(), _FakeCommExt()
    ctx = DistContext(rank=1, world_size=2, timeout_s=0.3)
    ctx.native, ctx.native_side = NativeComm(ext, 3, 2), NativeComm(ext_side, 4, 2)
    t0 = time.time()
    with pytest.raises(CollectiveError, match="did not complete"):
        ctx.wait_event(_NeverEvent())
    el = time.time() - t0
    assert 0.3 <= el < 5, el
    assert ext.aborted == [3] and ext_side.aborted == [4]      # both communicators aborted


def test_heartbeat_dead_peer_aborts_communicators_before_exit():
    from pytorch_dppo_amd.utils.heartbeat import Heartbeat
    calls = []

    class Store:
        def set(self, k, v):
            pass

    hb = Heartbeat(Store(), 0, 2, 0.1, 0.2, on_dead=None, abort=lambda msg: calls.append(msg))
    import pytorch_dppo_amd.utils.heartbeat as hbm
    real_exit = hbm.os._exit
    hbm.os._exit = lambda code: calls.append(code)
    try:
        hb._default_on_dead([1])
    finally:
        hbm.os._exit = real_exit
    assert len(calls) == 2 and "rank(s) [1]" in calls[0] and calls[1] == 75


def _worker_comm_create(rank, world, port, out_dir, mode):
    from pytorch_dppo_amd.parallel.dist import NativeComm
    _init(rank, world, port, timeout=30.0)
    ext = _FakeCommExt(fail_id=(mode == "id" and rank == 0), fail_init_rank=(1 if mode == "init" else None), rank=rank)
    nat = NativeComm.create(ext, rank, world, 5.0, device=torch.device("cpu"))
    with open(os.path.join(out_dir, f"c{rank}.txt"), "w") as f:
        f.write("none" if nat is None else "comm")


@pytest.mark.parametrize("mode", ["ok", "id", "init"])
def test_native_comm_creation_is_collective_safe(tmp_path, mode):
    """rank 0 failing to make the id, or one rank failing its init: EVERY rank falls back together
    (no rank left waiting in a broadcast or all-reduce the others skipped)"""
    codes = _join(_spawn(_worker_comm_create, 2, str(tmp_path), mode), 60)
    assert codes == [0, 0], codes
    got = [(tmp_path / f"c{r}.txt").read_text() for r in range(2)]
    assert got == (["comm", "comm"] if mode == "ok" else ["none", "none"]), got


def test_params_carry_the_execution_options():
    """the former DPPO_* environment switches are Params fields / CLI flags"""
    from pytorch_dppo_amd.config import params_from_args
    p = params_from_args(["--update-kernels", "tile", "--grad-comm", "process_group", "--dist-backend", "gloo",
                          "--fused-apply", "false", "--stats-stream", "on", "--wgrad-wgs", "128"])
    assert (p.update_kernels, p.grad_comm, p.dist_backend, p.fused_apply, p.stats_stream, p.wgrad_wgs) == \
        ("tile", "process_group", "gloo", False, "on", 128)
    with pytest.raises(ValueError):
        Params(update_kernels="bogus")
    assert Params().heartbeat_interval(1) == 0.0 and Params().heartbeat_interval(8) == 5.0
    assert Params(heartbeat_s=0).heartbeat_interval(8) == 0.0
