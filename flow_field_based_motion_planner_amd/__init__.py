"""MI355X-native batched flow-field motion-planning environment.

A drop-in for the `gym_ffmp` hot path of YoshitakaNagai/flow_field_based_motion_planner:
`FFMPVec` (N envs stepped by hand-written gfx950 HIP kernels through the C ABI
in include/ffmp.h) and the single-env `FFMP` class with the reference's
`rewarder`/`rewarder2`/`is_*` methods.  `gym_ffmp` (subpackage) mirrors the
reference's import paths; `install_gym_ffmp_alias()` makes `import gym_ffmp`
resolve to it.
"""
from .config import PRESETS, FFMPConfig, preset  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):  # lazy: torch / the HIP library load only when used
    if name == "FFMPVec":
        from .vec_env import FFMPVec
        return FFMPVec
    if name == "FFMP":
        from .env import FFMP
        return FFMP
    if name == "EpisodeTracker":
        from .episodes import EpisodeTracker
        return EpisodeTracker
    raise AttributeError(name)


def install_gym_ffmp_alias():
    """Make `import gym_ffmp` (and its submodules) resolve to this package's mirror."""
    import importlib
    import sys
    mods = ["gym_ffmp", "gym_ffmp.envs", "gym_ffmp.envs.ffmp", "gym_ffmp.envs.robot", "gym_ffmp.envs.robot.config"]
    for m in mods:
        sys.modules.setdefault(m, importlib.import_module(__name__ + "." + m))
    return sys.modules["gym_ffmp"]
