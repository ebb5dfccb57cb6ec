"""bench.py output contract (the driver parses this line): one JSON line from rank 0 with the
BASELINE metric, the whole-job value over all ranks, and the timing fields — at a tiny geometry,
on one GPU and as 2 ranks sharing it (gloo; RCCL refuses two ranks on one device, the driver's
N-GPU runs use RCCL through the same code path), launched by torchrun AND by a plain
``python bench.py --gpus 2`` (bench.py starts the ranks itself).  The world checks (WORLD_SIZE
must equal --gpus, one GPU per RCCL rank) run before any GPU call, so they are tested on CPU."""
import json
import os
import subprocess
import sys

import pytest


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--num-envs", "64", "--rollout-len", "4", "--num-epoch", "2", "--steps", "2", "--warmup", "1"]


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def _check(d: dict, n: int, variants: list) -> None:
    with open(os.path.join(ROOT, "BASELINE.json")) as f:
        base = json.load(f)
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["dtype"] == "fp32_3xbf16" and d["unit"] == "env_steps/s"
    rows = 64 * 4
    assert d["config"]["global_batch"] == rows * n and d["config"]["parallelism"] == f"dp{n}"
    # value = total env steps of all ranks / the max-over-ranks elapsed time
    assert d["value"] == pytest.approx(rows * n * 2 / (d["ms_per_step"] * 2 / 1e3), rel=1e-6)
    assert d["vs_baseline"] == pytest.approx(d["value"] / 1.6e3)
    assert sorted(d["variants"]) == sorted(variants)


@pytest.mark.gpu
def test_bench_json_line_one_gpu():
    from pytorch_dppo_amd.runtime.launcher import free_port
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))   # its world-1 RCCL group
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "1", *TINY, "--variants", "bf16"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_json_line(r.stdout), 1, ["bf16"])


@pytest.mark.gpu
def test_bench_json_line_two_ranks():
    from pytorch_dppo_amd.runtime.launcher import free_port
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", *TINY,
                        "--variants", "", "--verify-sync", "--dist-backend", "gloo"], cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    _check(_json_line(r.stdout), 2, [])
    assert "replicas_in_sync True" in r.stderr


@pytest.mark.gpu
def test_plain_bench_gpus_two_launches_two_ranks():
    """the driver's form `python bench.py --gpus N` (no torchrun): bench.py starts N ranks itself"""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", *TINY, "--variants", "", "--verify-sync",
                        "--dist-backend", "gloo"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    _check(d, 2, [])
    assert d["config"]["dist_backend"] == "gloo"
    assert "replicas_in_sync True" in r.stderr
    assert "launching 2 ranks" in r.stderr


@pytest.mark.gpu
def test_bench_one_gpu_reports_rccl_world():
    from pytorch_dppo_amd.runtime.launcher import free_port
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    r = subprocess.run([sys.executable, "bench.py", *TINY, "--variants", ""], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["config"]["rccl_world_size"] == 1 and d["config"]["dist_backend"] == "nccl"


def _bench_fails(args, extra_env):
    env = dict(os.environ, **extra_env)
    r = subprocess.run([sys.executable, "bench.py", *args, *TINY], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")], "no JSON line on a refused run"
    return r.stderr


def test_bench_refuses_world_size_mismatch():
    """a torchrun world of 2 launched as --gpus 4 must not be reported as 4 GPUs (CPU: the check
    runs before any GPU call)"""
    err = _bench_fails(["--gpus", "4"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0",
                                         "LOCAL_WORLD_SIZE": "2"})
    assert "WORLD_SIZE=2 but --gpus 4" in err


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """RCCL needs one GPU per local rank: on a box with fewer visible GPUs, a torchrun world and
    the plain --gpus N form (whose parent makes no HIP call: its ranks check) both exit non-zero
    without a JSON line, before any GPU work"""
    import torch
    n = max(2, torch.cuda.device_count() + 1)
    err = _bench_fails(["--gpus", str(n), "--dist-backend", "nccl"], {"WORLD_SIZE": str(n), "RANK": "0",
                                                                      "LOCAL_RANK": "0", "LOCAL_WORLD_SIZE": str(n)})
    assert "visible GPU" in err
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(n), *TINY], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "visible GPU" in r.stderr and f"launching {n} ranks" in r.stderr
