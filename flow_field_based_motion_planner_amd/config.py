"""FFMPConfig — the one POD-like configuration of the batched FFMP environment.

Reference constants it carries (YoshitakaNagai/flow_field_based_motion_planner):
  MAP_RESOLUTION 0.05, ROBOT_RSIZE 0.13, GOAL_THRESHOLHD 0.5, MAP_GRID_NUM 100,
  MAP_RANGE 5.0                       src/gym_ffmp/envs/ffmp.py:14-19
  MAX_STEPS 200                       src/train.py:60
  RobotAction.cmd[28]                 src/gym_ffmp/envs/robot/config.py:25-55
Everything else (dt, world size, obstacle model, potential-field constants,
lidar) has no reference implementation (Gazebo / external BEV nodes)
and is this framework's own specification — see DESIGN.md §SPEC.

This module is pure host logic (no torch, no GPU) so it is testable on CPU.
"""
from __future__ import annotations

import dataclasses
import math
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

COLLIDE_FOOTPRINT = 1
COLLIDE_LIDAR = 2
MAX_OBST = 64
MAX_FOOT = 128
MAX_BEAMS = 1024
N_ACTIONS = 28
REC_HDR = 16

# RobotAction.cmd (config.py:28-55) as literals: cmd[7*vi + wi] = (CMD_V[vi], CMD_W[wi]).
CMD_V = (0.0, 0.2, 0.4, 0.6)
CMD_W = (-0.6, -0.4, -0.2, 0.0, 0.2, 0.4, 0.6)


def action_table() -> List[Tuple[float, float]]:
    return [(v, w) for v in CMD_V for w in CMD_W]


def footprint_offsets(grid: int, res: float = 0.05, robot_r: float = 0.13) -> List[Tuple[int, int]]:
    """robot_grids of FFMP.is_collision (ffmp.py:87-94), generalised to any G.

    Cell (i, j) belongs to the footprint iff
        sqrt(pow(i*res - 0.5*R, 2) + pow(j*res - 0.5*R, 2)) <= robot_r,  R = G*res,
    evaluated in float64 exactly as the reference does (for G=100, R = 5.0 =
    MAP_RANGE).  Returned as offsets from (G//2, G//2), in the reference's
    (i, j) scan order.  Only a window around the centre can qualify.
    """
    map_range = grid * res
    c = grid // 2
    w = int(math.ceil(robot_r / res)) + 2
    out = []
    for i in range(max(0, c - w), min(grid, c + w + 1)):
        for j in range(max(0, c - w), min(grid, c + w + 1)):
            xp = math.pow(i * res - 0.5 * map_range, 2)
            yp = math.pow(j * res - 0.5 * map_range, 2)
            if math.sqrt(xp + yp) <= robot_r:
                out.append((i - c, j - c))
    return out


def beam_table(n_beams: int) -> np.ndarray:
    """(L, 2) float64 {cos, sin} of beam angles -pi + l*2pi/L (robot frame)."""
    out = np.zeros((n_beams, 2), dtype=np.float64)
    if n_beams:
        step = 2.0 * math.pi / n_beams
        for l in range(n_beams):
            th = -math.pi + l * step
            out[l, 0] = math.cos(th)
            out[l, 1] = math.sin(th)
    return out


@dataclass
class FFMPConfig:
    grid: int = 100                 # G (MAP_GRID_NUM, ffmp.py:15)
    n_obst: int = 4                 # K
    n_beams: int = 180              # L (0 disables lidar)
    max_steps: int = 200            # MAX_STEPS (train.py:60)
    moving: bool = False
    autoreset: bool = True
    collide_mode: Optional[int] = None  # default: footprint | (lidar if L > 0)
    res: float = 0.05               # MAP_RESOLUTION (ffmp.py:18)
    dt: float = 0.1                 # s per env step (SPEC)
    robot_r: float = 0.13           # ROBOT_RSIZE (ffmp.py:17)
    goal_thr: float = 0.5           # GOAL_THRESHOLHD (ffmp.py:19)
    world_half: Optional[float] = None   # default G*res (world side 2*G*res)
    lidar_max: Optional[float] = None    # default G*res/2
    goal_min: float = 1.0
    goal_max: Optional[float] = None     # default G*res/2
    obst_rmin: float = 0.10
    obst_rmax: float = 0.30
    obst_vmax: float = 0.5
    start_clear: float = 0.5
    goal_clear: float = 0.5
    k_att: float = 1.0
    k_rep: float = 0.1
    rho0: float = 0.5
    rho_min: Optional[float] = None      # default res/2
    cull_margin: float = 0.1
    flow: bool = False              # also raster the BEV motion-flow planes
    seed: int = 0

    # ---- derived -----------------------------------------------------------
    def __post_init__(self):
        self.validate()

    def validate(self):
        G = self.grid
        if G < 8 or G > 4096 or G % 4:
            raise ValueError(f"grid must be a multiple of 4 in [8, 4096], got {G}")
        if not 0 <= self.n_obst <= MAX_OBST:
            raise ValueError(f"n_obst must be in [0, {MAX_OBST}], got {self.n_obst}")
        if not 0 <= self.n_beams <= MAX_BEAMS:
            raise ValueError(f"n_beams must be in [0, {MAX_BEAMS}], got {self.n_beams}")
        if self.res <= 0 or self.dt < 0:
            raise ValueError("res must be > 0 and dt >= 0")
        if not 0 <= self.seed < 2 ** 64:
            raise ValueError("seed must fit in uint64")
        if len(self.footprint) > MAX_FOOT:
            raise ValueError("footprint too large")

    @property
    def W(self) -> float:
        return self.grid * self.res if self.world_half is None else float(self.world_half)

    @property
    def lidar_range(self) -> float:
        return 0.5 * self.grid * self.res if self.lidar_max is None else float(self.lidar_max)

    @property
    def goal_hi(self) -> float:
        return 0.5 * self.grid * self.res if self.goal_max is None else float(self.goal_max)

    @property
    def rho_lo(self) -> float:
        return 0.5 * self.res if self.rho_min is None else float(self.rho_min)

    @property
    def mode(self) -> int:
        if self.collide_mode is not None:
            return int(self.collide_mode)
        return COLLIDE_FOOTPRINT | (COLLIDE_LIDAR if self.n_beams > 0 else 0)

    @property
    def footprint(self) -> List[Tuple[int, int]]:
        return footprint_offsets(self.grid, self.res, self.robot_r)

    def f32_constants(self) -> Dict[str, np.float32]:
        """The float32 raster constants, each = (float)(double expression)."""
        f = np.float32
        return {
            "res_f": f(self.res),
            "half_f": f(0.5 * (self.grid * self.res)),
            "world_half_f": f(self.W),
            "half_ka_f": f(0.5 * self.k_att),
            "half_kr_f": f(0.5 * self.k_rep),
            "rho0_f": f(self.rho0),
            "inv_rho0_f": f(1.0 / self.rho0),
            "rho_min_f": f(self.rho_lo),
            "inv_2res_f": f(1.0 / (2.0 * self.res)),
            "cull_margin_f": f(self.cull_margin),
        }

    def record_len(self) -> int:
        return REC_HDR + 12 * self.n_obst

    def replace(self, **kw) -> "FFMPConfig":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)


# Benchmark configurations (BASELINE.json:configs; SURVEY §8 "Config shorthand").
# n_envs is the TOTAL env count; gpus the GPU count the config is quoted on.
PRESETS: Dict[str, dict] = {
    "C1": dict(n_envs=1, gpus=0, cfg=dict(grid=64, n_obst=4, moving=False, n_beams=0)),
    "C2": dict(n_envs=4096, gpus=1, cfg=dict(grid=128, n_obst=8, moving=False, n_beams=0)),
    "C3": dict(n_envs=32768, gpus=1, cfg=dict(grid=256, n_obst=16, moving=True, n_beams=180)),
    "C4": dict(n_envs=65536, gpus=8, cfg=dict(grid=256, n_obst=16, moving=True, n_beams=180)),
    "C5": dict(n_envs=131072, gpus=8, cfg=dict(grid=512, n_obst=32, moving=True, n_beams=360)),
}


def preset(name: str, **overrides) -> FFMPConfig:
    if name not in PRESETS:
        raise KeyError(f"unknown preset {name!r}; known: {sorted(PRESETS)}")
    kw = dict(PRESETS[name]["cfg"])
    kw.update(overrides)
    return FFMPConfig(**kw)


def bytes_per_env_step(cfg: FFMPConfig, potential: bool = True, window: int = 2,
                       seamless: bool = False, obs_format: str = "f32") -> Dict[str, int]:
    """Algorithmic HBM bytes of one env step.

    raster kernel: writes the new float32 frame of state_m (4 G^2), the older one too on the
    steps where the frame window wraps (every W-1 steps; every step for W = 2; never with the
    seamless ring) — plus, not
    counted here, the older frame of each env reset on the other steps —, the float32 potential
    plane (4 G^2) and, with cfg.flow, the two float32 flow planes (8 G^2); reads the raster
    record (64 + 48 K).  state kernel: reads/writes pose, goal, d0, t, episode, obstacles and
    writes the small obs, lidar and the record.  obs_format "u8f16" (FFMPVec): 1-byte frames and
    a 2-byte potential plane (and 2-byte flow planes) instead.
    """
    G2 = cfg.grid * cfg.grid
    K, L = cfg.n_obst, cfg.n_beams
    rec = 4 * cfg.record_len()
    fb, pb = {"f32": (4, 4), "u8f16": (1, 2)}[obs_format]
    frames = fb * G2 + (0 if seamless and window > 2 else (fb * G2) // (max(int(window), 2) - 1))
    raster = frames + (pb * G2 if potential else 0) + (2 * pb * G2 if cfg.flow else 0) + rec
    state_rw = 2 * (24 + 16 + 8 + 4 + 4 + 40 * K)  # pose, goal, d0, t, episode, obst(32)+r(8)
    small_obs = 4 * (2 + 2 + 1 + 2) + 4 * L + rec + 8 + 4 + 4  # g, v, t, grad, lidar, record, action, reward, flags
    return {"raster": raster, "state": state_rw + small_obs, "total": raster + state_rw + small_obs}
