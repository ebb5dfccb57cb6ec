"""Host-side plan of the grouped wgrad launch (pytorch_dppo_amd/runtime/engine_hip.py
wgrad_tiles): every layer's [fan_out][fan_in + 1] gradient is covered exactly once by tiles the
kernel accepts (csrc/wgrad.hip: nq*kq <= 8 waves, nq + kq <= 6 fragment slots, tiles inside the
128-row padded operand buffers).  CPU only — the kernel itself is checked against autograd in
tests/test_gpu_kernels.py."""
import pytest
import torch

from pytorch_dppo_amd.runtime.engine_hip import WT, wgrad_tiles

# (fan_out, fan_in) of the six layers for the reference envs' obs / act dims
LAYERS = {
    "Humanoid-v2": [(100, 376), (100, 100), (17, 100), (500, 376), (100, 500), (1, 100)],
    "HalfCheetah-v2": [(100, 17), (100, 100), (6, 100), (500, 17), (100, 500), (1, 100)],
    "InvertedPendulum-v1": [(100, 4), (100, 100), (1, 100), (500, 4), (100, 500), (1, 100)],
}


def _r(x, m):
    return -(-x // m) * m


@pytest.mark.parametrize("env", sorted(LAYERS))
def test_tiles_cover_each_gradient_once(env):
    for li, (n, fan_in) in enumerate(LAYERS[env]):
        k = fan_in + 1
        cover = torch.zeros(_r(n, 64), _r(k, 64), dtype=torch.int32)
        for (tl, n0, k0, nq, kq) in wgrad_tiles(li, n, k):
            assert tl == li
            assert nq >= 1 and kq >= 1 and nq * kq <= 8 and nq + kq <= 6
            assert n0 % 64 == 0 and k0 % 64 == 0
            # operand buffers hold _r(rows, WT) rows (engine_hip: g_rows / x_rows)
            assert n0 + 64 * nq <= _r(n, WT) and k0 + 64 * kq <= _r(k, WT)
            cover[n0:n0 + 64 * nq, k0:k0 + 64 * kq] += 1
        assert bool((cover == 1).all()), (env, li)


def test_humanoid_value_fc1_streams_fewer_rows_than_square_tiles():
    tiles = wgrad_tiles(3, 500, 377)
    rows_per_step = sum(64 * (nq + kq) for (_, _, _, nq, kq) in tiles)
    square = (_r(500, 128) // 128) * (_r(377, 128) // 128) * 256   # 128x128 tiles
    assert rows_per_step == 2304 and rows_per_step < square
