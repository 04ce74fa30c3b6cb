"""FFMP — the single-env `gym.Env` surface of gym_ffmp, backed by the HIP kernels.

Mirrors src/gym_ffmp/envs/ffmp.py:22-188 of the reference
(YoshitakaNagai/flow_field_based_motion_planner):

  attributes / spaces         ffmp.py:25-64  (action Box [0,-.6]..[.6,.6]; obs Dict
                              local_map int32 (G,G,1), relative_goal, velocity)
  is_collision(local_map)     ffmp.py:85-105  -> ffmp_footprint_collision kernel
  is_collision2(scan_data)    ffmp.py:108-117 -> ffmp_scan_collision_f64 kernel (+ the
                              reference's "!!!..." banner on a hit, unless verbose=False)
  is_goal(d)                  ffmp.py:120-127 -> ffmp_reward_done kernel
  reward_calculator(...)      ffmp.py:130-157 -> ffmp_reward_done kernel; keeps the
                              reference's MODULE-GLOBAL pre_relative_goal_dist (shared by
                              every FFMP instance, NameError before the first is_first)
  is_done(col, goal)          ffmp.py:160-164 (host boolean)
  rewarder / rewarder2        ffmp.py:167-188 -> one ffmp_reward_done launch each

New (the reference's reset is commented out, ffmp.py:77-83, and it has no step):
  reset(seed=None) -> obs,  step(action_id) -> (obs, reward, done, info)  [gym 0.17/0.18
  4-tuple API], run by a 1-env FFMPVec with autoreset off.  In this gym surface the
  episode-start distance d0 is per instance (kept on the device), not the module global.

Every compute path goes through libffmp; without it (or without a GPU) calls raise.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional

import numpy as np
import torch

from . import _abi
from ._spaces import Box, Dict as DictSpace, GymEnvBase
from .config import CMD_V, CMD_W, FFMPConfig

MAP_RANGE = 5.0          # ffmp.py:14
MAP_GRID_NUM = 100       # ffmp.py:15
MAP_CHANNELS = 1         # ffmp.py:16
ROBOT_RSIZE = 0.13       # ffmp.py:17
MAP_RESOLUTION = 0.05    # ffmp.py:18
GOAL_THRESHOLHD = 0.5    # ffmp.py:19 (sic)
_BANNER = "!" * 43       # ffmp.py:114

# ffmp.py:139 `global pre_relative_goal_dist` — shared by all instances.
_PRE_RELATIVE_GOAL_DIST: Optional[float] = None


def _reset_global_d0():
    global _PRE_RELATIVE_GOAL_DIST
    _PRE_RELATIVE_GOAL_DIST = None


def default_config() -> FFMPConfig:
    """The reference's 100x100 / 5 m map with a 180-beam lidar, 4 static discs."""
    return FFMPConfig(grid=MAP_GRID_NUM, n_obst=4, n_beams=180, moving=False, autoreset=False)


class FFMP(GymEnvBase):
    metadata = {"render.modes": []}

    def __init__(self, config: Optional[FFMPConfig] = None, device=None, verbose: bool = True):
        self.cfg = config if config is not None else default_config()
        self.verbose = verbose
        self._device = device
        from .gym_ffmp.envs.robot.config import RobotAction
        # [1] action_space (ffmp.py:29-32)
        self.action = RobotAction()
        self.action_low = np.array([self.action.cmd[0].linear_v, self.action.cmd[0].angular_v])
        self.action_high = np.array([self.action.cmd[27].linear_v, self.action.cmd[27].angular_v])
        self.action_space = Box(self.action_low, self.action_high, dtype=np.float32)
        # [2] observation_space (ffmp.py:34-57)
        self.map_grid_num = self.cfg.grid
        self.map_grid_size = self.cfg.res
        self.map_range = MAP_RANGE if self.cfg.grid == MAP_GRID_NUM else self.cfg.grid * self.cfg.res
        self.map_channels = MAP_CHANNELS
        self.map_low = np.full((self.map_grid_num, self.map_grid_num, self.map_channels), 0)
        self.map_high = np.full((self.map_grid_num, self.map_grid_num, self.map_channels), 255)
        self.goal_low = np.array([0.0, 0.0])
        self.goal_high = np.array([math.sqrt(2.0) * self.map_range, math.pi])
        self.velocity_low = self.action_low
        self.velocity_high = self.action_high
        self.robot_rsize = self.cfg.robot_r
        self.collision_low = False
        self.collision_high = True
        self.observation = np.array([self.goal_high, self.action_low])
        self.observation_space = DictSpace({
            "local_map": Box(self.map_low, self.map_high, dtype=np.int32),
            "relative_goal": Box(self.goal_low, self.goal_high, dtype=np.float32),
            "velocity": Box(self.velocity_low, self.velocity_high, dtype=np.float32)})
        self.state_space = DictSpace(dict(self.observation_space.spaces))
        self.robot_grids = []
        self._vec = None
        self._needs_reset = True

    # ------------------------------------------------------------- plumbing
    @property
    def device(self) -> torch.device:
        if self._device is None:
            if not torch.cuda.is_available():
                raise _abi.FFMPBackendError("FFMP needs a ROCm GPU; there is no CPU path")
            self._device = torch.device("cuda", torch.cuda.current_device())
        return torch.device(self._device)

    def _legacy_cfg(self, grid: int):
        """ctypes cfg for the legacy kernels: the footprint of THIS instance's map
        attributes (ffmp.py:87-94 reads self.map_grid_num / map_grid_size / map_range
        / robot_rsize) as absolute cells, re-centred on the given map's width."""
        if grid % 4 or grid < 8:
            raise ValueError(f"local map width must be a multiple of 4 and >= 8, got {grid}")
        cells = []
        half = 0.5 * self.map_range
        for i in range(self.map_grid_num):
            xp = math.pow(i * self.map_grid_size - half, 2)
            if math.sqrt(xp) > self.robot_rsize:
                continue
            for j in range(self.map_grid_num):
                yp = math.pow(j * self.map_grid_size - half, 2)
                if math.sqrt(xp + yp) <= self.robot_rsize:
                    cells.append((i, j))
        self.robot_grids = [np.array([i, j]) for i, j in cells]
        cfg = self.cfg.replace(grid=grid, n_beams=0, n_obst=0)
        c = _abi.make_cfg(cfg)
        c.n_foot = len(cells)
        for k, (i, j) in enumerate(cells):
            c.foot_di[k], c.foot_dj[k] = i - grid // 2, j - grid // 2
        c.robot_r = float(self.robot_rsize)
        return c

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def _reward_done(self, rel_goal, is_first: bool, d0: float, scan=None, local_map=None,
                     collide_in=None, goal_in=None):
        lib = _abi.load()
        dev = self.device
        f64 = dict(dtype=torch.float64, device=dev)
        u8 = dict(dtype=torch.uint8, device=dev)
        grid = self.cfg.grid
        m_t = None
        if local_map is not None:
            m = np.asarray(local_map)
            if m.ndim == 3:
                m = m[:, :, 0]
            if m.ndim != 2 or m.shape[0] != m.shape[1]:
                raise ValueError(f"local_map must be (G,G) or (G,G,1), got {np.shape(local_map)}")
            grid = m.shape[0]
            m_t = torch.as_tensor(np.ascontiguousarray(m, dtype=np.float32)).to(dev)
        cfg_c = self._legacy_cfg(grid)
        s_t = None
        L = 0
        if scan is not None:
            vals = np.array([0.0 if v is None else float(v) for v in scan], dtype=np.float64)
            L = len(vals)
            s_t = torch.as_tensor(vals).to(dev) if L else None
        rg = torch.tensor([float(rel_goal[0]), float(rel_goal[1]) if len(rel_goal) > 1 else 0.0], **f64)
        first = torch.tensor([1 if is_first else 0], **u8)
        d0_t = torch.tensor([d0], **f64)
        ci = None if collide_in is None else torch.tensor([1 if collide_in else 0], **u8)
        gi = None if goal_in is None else torch.tensor([1 if goal_in else 0], **u8)
        reward = torch.empty(1, **f64)
        done, goal, col = (torch.empty(1, **u8) for _ in range(3))
        p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
        _abi.check(lib.ffmp_reward_done(C.byref(cfg_c), 1, p(s_t), L, p(m_t), grid * grid, p(ci), p(gi),
                                        rg.data_ptr(), first.data_ptr(), d0_t.data_ptr(), reward.data_ptr(),
                                        done.data_ptr(), goal.data_ptr(), col.data_ptr(), self._stream()),
                   "ffmp_reward_done")
        out = torch.cat([reward, d0_t, done.double(), goal.double(), col.double()]).cpu().numpy()
        return float(out[0]), float(out[1]), bool(out[2]), bool(out[3]), bool(out[4])

    # ---------------------------------------------------- reference methods
    def is_collision(self, local_map_info) -> bool:
        m = np.asarray(local_map_info)
        if m.ndim == 3:
            m = m[:, :, 0]
        grid = m.shape[0]
        cfg_c = self._legacy_cfg(grid)
        dev = self.device
        m_t = torch.as_tensor(np.ascontiguousarray(m, dtype=np.float32)).to(dev)
        col = torch.empty(1, dtype=torch.uint8, device=dev)
        _abi.check(_abi.load().ffmp_footprint_collision(C.byref(cfg_c), 1, m_t.data_ptr(), grid * grid,
                                                        col.data_ptr(), self._stream()), "ffmp_footprint_collision")
        return bool(col.item())

    def is_collision2(self, scan_data) -> bool:
        vals = np.array([0.0 if v is None else float(v) for v in scan_data], dtype=np.float64)
        if len(vals) == 0:
            return False
        dev = self.device
        s_t = torch.as_tensor(vals).to(dev)
        col = torch.empty(1, dtype=torch.uint8, device=dev)
        _abi.check(_abi.load().ffmp_scan_collision_f64(1, len(vals), s_t.data_ptr(), float(ROBOT_RSIZE),
                                                       col.data_ptr(), None, self._stream()), "ffmp_scan_collision")
        hit = bool(col.item())
        if hit and self.verbose:
            print(_BANNER)
        return hit

    def is_goal(self, cur_relative_goal_dist) -> bool:
        _, _, _, goal, _ = self._reward_done([cur_relative_goal_dist, 0.0], True, 0.0, collide_in=False)
        return goal

    def reward_calculator(self, relative_goal_info, is_collision, is_goal, is_first):
        global _PRE_RELATIVE_GOAL_DIST
        if is_first:
            _PRE_RELATIVE_GOAL_DIST = relative_goal_info[0]
        if _PRE_RELATIVE_GOAL_DIST is None:
            raise NameError("name 'pre_relative_goal_dist' is not defined")
        r, _, _, _, _ = self._reward_done(relative_goal_info, False, float(_PRE_RELATIVE_GOAL_DIST),
                                          collide_in=bool(is_collision), goal_in=bool(is_goal))
        return r if is_goal or not isinstance(relative_goal_info[0], np.floating) else np.float64(r)

    def is_done(self, is_collision, is_goal) -> bool:
        return bool(is_collision or is_goal)

    def _legacy_d0(self, relative_goal_info, is_first):
        global _PRE_RELATIVE_GOAL_DIST
        if not is_first and _PRE_RELATIVE_GOAL_DIST is None:
            raise NameError("name 'pre_relative_goal_dist' is not defined")
        return 0.0 if is_first else float(_PRE_RELATIVE_GOAL_DIST)

    def rewarder(self, local_map_info, relative_goal_info, is_first):
        global _PRE_RELATIVE_GOAL_DIST
        d0 = self._legacy_d0(relative_goal_info, is_first)
        r, d0n, done, goal, col = self._reward_done(relative_goal_info, bool(is_first), d0, local_map=local_map_info)
        if is_first:
            _PRE_RELATIVE_GOAL_DIST = relative_goal_info[0]
        return (r if goal or not isinstance(relative_goal_info[0], np.floating) else np.float64(r)), done

    def rewarder2(self, scan_data, relative_goal_info, is_first):
        global _PRE_RELATIVE_GOAL_DIST
        d0 = self._legacy_d0(relative_goal_info, is_first)
        r, d0n, done, goal, col = self._reward_done(relative_goal_info, bool(is_first), d0, scan=scan_data)
        if is_first:
            _PRE_RELATIVE_GOAL_DIST = relative_goal_info[0]
        if col and self.verbose:
            print(_BANNER)
        return (r if goal or not isinstance(relative_goal_info[0], np.floating) else np.float64(r)), done, goal

    # ------------------------------------------------------------- gym API
    def _vec_env(self):
        if self._vec is None:
            from .vec_env import FFMPVec
            self._vec = FFMPVec(1, self.cfg.replace(autoreset=False), device=self.device)
        return self._vec

    def _obs(self):
        v = self._vec
        m = v.state_m[0, 1].to(torch.int32).unsqueeze(-1)
        return {"local_map": m.cpu().numpy(),
                "relative_goal": v.state_g[0].cpu().numpy().astype(np.float32),
                "velocity": v.state_v[0].cpu().numpy().astype(np.float32)}

    def _extras(self):
        v = self._vec
        d = {"state_m": v.state_m[0:1].cpu().numpy(), "state_t": v.state_t[0:1].cpu().numpy(),
             "grad": v.grad[0].cpu().numpy()}
        if v.potential is not None:
            d["potential"] = v.potential[0].cpu().numpy()
        if v.lidar is not None:
            d["lidar"] = v.lidar[0].cpu().numpy()
        return d

    def reset(self, seed: Optional[int] = None):
        v = self._vec_env()
        v.reset(seed=seed)
        self._needs_reset = False
        return self._obs()

    def step(self, action):
        if self._needs_reset:
            raise RuntimeError("call reset() before step() (and after an episode ends)")
        a = int(action)
        if not 0 <= a < 28:
            raise IndexError(f"action id {a} out of range 0..27 (RobotAction.cmd has 28 entries)")
        v = self._vec
        v.step(torch.tensor([a], dtype=torch.int64, device=v.device))
        reward = float(v.reward[0].item())
        done = bool(v.done[0].item())
        info = {"is_goal": bool(v.is_goal[0].item()), "collision": bool(v.collision[0].item()),
                "truncated": bool(v.truncated[0].item())}
        info.update(self._extras())
        if done:
            self._needs_reset = True
        return self._obs(), reward, done, info

    def render(self, mode="human"):
        return None

    def close(self):
        self._vec = None

    def seed(self, seed=None):
        self.cfg = self.cfg.replace(seed=int(seed or 0))
        return [self.cfg.seed]


def commander_table():
    """(v, w) of every action id (config.py:57-58 commander)."""
    return [(v, w) for v in CMD_V for w in CMD_W]
