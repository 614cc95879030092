"""Env ids of the reference (gym_futbol/__init__.py:3-28) and `make()`.

    make("Futbol2v2-v1")                 -> Futbol(number_of_player=2)     (like gym.make)
    make("Futbol2v2-v1", num_envs=65536) -> FutbolVecEnv of 65536 envs on the GPU
    make("gym_futbol:Futbol-v0", ...)    -> the "module:id" form resolves the same ids

If gym is importable, importing the package also registers the ids with gym
(entry points are the single-env facades), so `gym.make('Futbol2v2-v1')` works.
"""
from .vec_env import FutbolVecEnv

ENV_SPECS = {
    "Futbol-v0": ("v0", {}),
    "Futbol-extrahard-v0": None,  # registered by the reference, but its class does not exist
    "Futbol-v1": ("v1", {"number_of_player": 10}),
    "Futbol2v2-v1": ("v1", {"number_of_player": 2}),
    "Futbol5v5-v1": ("v1", {"number_of_player": 5}),
}


def spec(env_id):
    if ":" in env_id:
        env_id = env_id.split(":", 1)[1]
    if env_id not in ENV_SPECS:
        raise KeyError("No registered env with id: %s" % env_id)
    s = ENV_SPECS[env_id]
    if s is None:
        raise AttributeError("entry point gym_futbol.envs:FutbolExtraHardEnv does not exist in the reference")
    return s


def make(env_id, num_envs=None, device="cuda", seed=0, env_id_base=0, **kwargs):
    kind, defaults = spec(env_id)
    kw = dict(defaults)
    kw.update(kwargs)
    if num_envs is None:
        if kind == "v1":
            from .envs_v1 import Futbol
            return Futbol(device=device, seed=seed, env_id=env_id_base, **kw)
        from .envs import FutbolEnv
        return FutbolEnv(device=device, seed=seed, env_id=env_id_base, **kw)
    return FutbolVecEnv(kind, num_envs, device=device, seed=seed, env_id_base=env_id_base, **kw)


def register_with_gym():  # pragma: no cover - gym is absent in this image
    try:
        from gym.envs.registration import register
    except Exception:  # noqa: BLE001
        return False
    for env_id, s in ENV_SPECS.items():
        if s is None:
            continue
        kind, kw = s
        entry = "gym_futbol_amd.envs_v1:Futbol" if kind == "v1" else "gym_futbol_amd.envs:FutbolEnv"
        try:
            register(id=env_id, entry_point=entry, kwargs=kw)
        except Exception:  # noqa: BLE001 - already registered (e.g. by the reference package)
            pass
    return True
