"""gym_futbol_amd -- MI355X-native vectorised gym-futbol envs.

The reference's gym ids and APIs (gym_futbol/__init__.py, envs_v1/futbol_env.py,
envs/futbol_env.py) backed by hand-written HIP kernels for gfx950
(libfutbol_amd.so, C ABI in include/futbol.h).  See DESIGN.md.
"""
from ._native import LIB_PATH, NativeError, load as load_native
from .registration import ENV_SPECS, make, register_with_gym, spec
from .vec_env import FutbolVecEnv, SB3VecEnv
from .envs_v1 import Futbol
from .envs import FutbolEnv
from .evaluation import evaluate_policy
from .policy import SB2MlpPolicy
from .ppo import PPO2, ActorCritic
from .a2c import A2C
from .monitor import VecMonitor, EvalCallback, load_results

__all__ = ["make", "spec", "ENV_SPECS", "FutbolVecEnv", "SB3VecEnv", "Futbol", "FutbolEnv", "NativeError",
           "LIB_PATH", "load_native",
           "evaluate_policy", "SB2MlpPolicy", "PPO2", "A2C", "ActorCritic", "VecMonitor", "EvalCallback", "load_results"]

register_with_gym()
