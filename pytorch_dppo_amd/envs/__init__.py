from .registry import EnvSpec, get_spec, host_spec, known_envs, KIND_HOST, KIND_PENDULUM, KIND_SYNTHETIC
from .vec_env import VecEnv, SyntheticEnv, PendulumEnv, make_vec_env
from .gym_adapter import GymVecEnv, gym_available, register_env

__all__ = ["EnvSpec", "get_spec", "host_spec", "known_envs", "KIND_HOST", "KIND_PENDULUM", "KIND_SYNTHETIC",
           "VecEnv", "SyntheticEnv", "PendulumEnv", "make_vec_env", "GymVecEnv", "gym_available", "register_env"]
