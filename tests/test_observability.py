"""Heartbeat failure detection, learning-curve CSV, torch.profiler window and the finite-check
debug mode.  CPU only."""
import csv
import json
import os
import time
from datetime import timedelta

import pytest
import torch
import torch.distributed as dist

from pytorch_dppo_amd.config import dppo_preset
from pytorch_dppo_amd.parallel.dist import DistContext
from pytorch_dppo_amd.runtime.launcher import free_port, run_worker
from pytorch_dppo_amd.utils.heartbeat import Heartbeat


def _store_pair():
    port = free_port()
    server = dist.TCPStore("127.0.0.1", port, is_master=True, timeout=timedelta(seconds=10),
                           wait_for_workers=False)
    client = dist.TCPStore("127.0.0.1", port, is_master=False, timeout=timedelta(seconds=10))
    return server, client


def _wait(pred, seconds):
    t0 = time.time()
    while time.time() - t0 < seconds:
        if pred():
            return True
        time.sleep(0.05)
    return pred()


def test_heartbeat_reports_a_silent_rank_once():
    s0, s1 = _store_pair()
    seen = []
    hb0 = Heartbeat(s0, 0, 2, interval_s=0.1, timeout_s=0.6, on_dead=seen.append).start()
    hb1 = Heartbeat(s1, 1, 2, interval_s=0.1, timeout_s=0.6, on_dead=lambda d: None).start()
    time.sleep(0.8)
    assert seen == []                      # both alive: no false positive
    hb1.stop(done=False)                   # rank 1 "crashes": stops beating, never writes done
    assert _wait(lambda: seen == [[1]], 3.0), seen
    time.sleep(0.5)
    assert seen == [[1]]                   # reported once
    hb0.stop()


def test_heartbeat_ignores_a_rank_that_finished():
    s0, s1 = _store_pair()
    seen = []
    hb0 = Heartbeat(s0, 0, 2, interval_s=0.1, timeout_s=0.5, on_dead=seen.append).start()
    hb1 = Heartbeat(s1, 1, 2, interval_s=0.1, timeout_s=0.5, on_dead=lambda d: None).start()
    time.sleep(0.3)
    hb1.stop(done=True)
    time.sleep(1.2)
    assert seen == []
    hb0.stop()


def test_csv_and_profiler_trace(tmp_path):
    p = dppo_preset(env_name="HalfCheetah-v2", num_processes=1, num_envs=8, exploration_size=64, batch_size=64,
                    num_epoch=2, hidden=(16, 16), max_iters=3, log_csv=str(tmp_path / "curve.csv"),
                    profile_dir=str(tmp_path / "prof"), profile_iters="1:2", check_finite=True)
    run_worker(p, DistContext(), evaluator=False, quiet=True)
    rows = list(csv.DictReader(open(tmp_path / "curve.csv")))
    assert [int(float(r["iteration"])) for r in rows] == [1, 2, 3]
    assert all(float(r["env_steps"]) > 0 for r in rows)
    trace = json.load(open(tmp_path / "prof" / "trace_rank0.json"))
    names = {e.get("name") for e in trace.get("traceEvents", [])}
    assert {"rollout", "update"} <= names     # PhaseTimer ranges are in the trace


def test_check_finite_names_the_failure():
    from pytorch_dppo_amd.runtime.worker import DPPOWorker
    p = dppo_preset(env_name="HalfCheetah-v2", num_processes=1, num_envs=8, exploration_size=64, batch_size=64,
                    num_epoch=1, hidden=(16, 16), check_finite=True)
    w = DPPOWorker(p, DistContext())
    w.iteration_step()
    with torch.no_grad():
        w.model.flat.data[5] = float("nan")
    with pytest.raises(FloatingPointError, match="non-finite"):
        w.iteration_step()
