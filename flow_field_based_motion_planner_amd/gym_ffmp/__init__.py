"""Mirror of the reference package `gym_ffmp` (src/gym_ffmp/__init__.py:1-6).

Registers FFMP-v0 with gym when gym is importable; `import gym_ffmp` works after
`flow_field_based_motion_planner_amd.install_gym_ffmp_alias()` (or with this
package's parent directory on sys.path)."""
from ._register import register_ffmp

register_ffmp()
from .envs.ffmp import FFMP  # noqa: E402,F401
