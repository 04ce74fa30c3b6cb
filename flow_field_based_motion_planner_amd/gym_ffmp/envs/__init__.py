from .ffmp import FFMP  # noqa: F401  (src/gym_ffmp/envs/__init__.py:1)
