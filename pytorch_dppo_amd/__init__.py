"""pytorch_dppo_amd — an MI355X-native Distributed PPO trainer.

Same capabilities as kibeomKim/Pytorch-DPPO (synchronous multi-worker PPO, GAE, shared
observation normalisation, diagonal-Gaussian tanh-MLP actor-critic, online evaluator,
single-process PPO), re-designed for MI355X: hand-written CDNA4 HIP kernels for the rollout,
value/GAE, fused loss forward/backward, wgrad and Adam; RCCL all-reduce over xGMI between
one process per GPU.  The importable package name uses an underscore; ``pytorch-dppo_amd``
is a symlink to it.
"""
from .config import Params, dppo_preset, ppo_preset  # noqa: F401

__version__ = "0.1.0"
