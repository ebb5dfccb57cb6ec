#!/usr/bin/env python3
"""Shim for the reference's single-process PPO program (``ppo.py``): PPO preset, 1 process.

Equivalent to ``python train.py --preset ppo [flags]``.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_dppo_amd.config import params_from_args  # noqa: E402
from pytorch_dppo_amd.runtime.launcher import launch  # noqa: E402

if __name__ == "__main__":
    launch(params_from_args(["--preset", "ppo"] + sys.argv[1:]))
