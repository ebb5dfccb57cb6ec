#!/usr/bin/env python3
"""Training entrypoint (north star: "train.py entrypoint").

    python train.py --preset dppo --env-name Pendulum-v0 --num-processes 2 --hidden 64,64
    python train.py --preset ppo  --env-name HalfCheetah-v2 --device gpu --num-envs 1024 --dtype bf16
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 train.py --device gpu --env-name Humanoid-v2 ...

``--preset dppo`` = reference ``main.py`` hyper-parameters (DPPO, N workers),
``--preset ppo``  = reference ``ppo.py`` hyper-parameters (single process).
Every ``Params`` field is a flag (``--gae-param``, ``--ent-coeff``, ``--update-treshold`` …).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_dppo_amd.config import params_from_args  # noqa: E402
from pytorch_dppo_amd.runtime.launcher import launch  # noqa: E402


def main(argv=None):
    params = params_from_args(argv)
    launch(params)


if __name__ == "__main__":
    main()
