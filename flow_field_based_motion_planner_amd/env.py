"""FFMP — the single-env `gym.Env` surface of gym_ffmp, backed by the HIP kernels.

Mirrors src/gym_ffmp/envs/ffmp.py:22-188 of the reference
(YoshitakaNagai/flow_field_based_motion_planner):

  attributes / spaces         ffmp.py:25-64  (action Box [0,-.6]..[.6,.6]; obs Dict
                              local_map int32 (G,G,1), relative_goal, velocity)
  is_collision(local_map)     ffmp.py:85-105  -> the footprint test of ffmp_reward_done
  is_collision2(scan_data)    ffmp.py:108-117 -> the lidar test of ffmp_reward_done (+ the
                              reference's "!!!..." banner on a hit, unless verbose=False)
  is_goal(d)                  ffmp.py:120-127 -> ffmp_reward_done kernel
  reward_calculator(...)      ffmp.py:130-157 -> ffmp_reward_done kernel; keeps the
                              reference's MODULE-GLOBAL pre_relative_goal_dist (shared by
                              every FFMP instance, NameError before the first is_first)
  is_done(col, goal)          ffmp.py:160-164 (host boolean)
  rewarder / rewarder2        ffmp.py:167-188 -> one ffmp_reward_done launch each
Each of these is ONE library call (ffmp_reward_done_packed): the inputs packed into a pinned host
buffer, one copy in, the kernel, one copy out, the stream synchronized; the footprint is cached per
(map attributes, width) instead of rebuilt over all G^2 cells per call (ffmp.py:87-94).

New (the reference's reset is commented out, ffmp.py:77-83, and it has no step):
  reset(seed=None) -> obs,  step(action_id) -> (obs, reward, done, info)  [gym 0.17/0.18
  4-tuple API], run by a 1-env FFMPVec with autoreset off.  In this gym surface the
  episode-start distance d0 is per instance (kept on the device), not the module global.

Every compute path goes through libffmp; without it (or without a GPU) calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
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
        self._cfg_cache = {}  # (map attributes, width) -> (ctypes cfg with the footprint, robot_grids)
        self._stage = None    # pinned host / device staging buffers of the legacy methods

    # ------------------------------------------------------------- plumbing
    @property
    def device(self) -> torch.device:
        if self._device is None:
            if not torch.cuda.is_available():
                raise _abi.FFMPBackendError("FFMP needs a ROCm GPU; there is no CPU path")
            self._device = torch.device("cuda", torch.cuda.current_device())
        return torch.device(self._device)

    def _legacy_cfg(self, shape):
        """(ctypes cfg, checked cells, complete) for the legacy kernels and a local map of `shape`
        (H, W).  The footprint is THIS instance's (ffmp.py:87-94 reads self.map_grid_num /
        map_grid_size / map_range / robot_rsize): ABSOLUTE cells (i, j) in the reference's list order,
        indexed into the given map as local_map_info[i, j] (ffmp.py:97-101) — whatever the map's
        width, and whether or not it equals map_grid_num.  The reference raises IndexError at the
        first cell outside the map that its loop reaches before a hit: the kernel checks the cells
        before that one (complete = False) and the caller raises when none of them is occupied.  The
        map is staged into a square plane of side `grid` (max(H, W) rounded up to the kernels' multiple
        of 4, >= 8; the padding is never read).  Built once per (attributes, shape) and cached (the
        reference rebuilds the list over all cells on every call; the attributes are public)."""
        H, W = int(shape[0]), int(shape[1])
        key = (H, W, self.map_grid_num, self.map_grid_size, self.map_range, self.robot_rsize, id(self.cfg))
        hit = self._cfg_cache.get(key)
        if hit is not None and hit[3] is self.cfg:  # (a config is replaced, never mutated: FFMPConfig.replace)
            self.robot_grids = hit[1]
            return hit[0], hit[2]  # (ctypes cfg, complete)
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
        k_oor = next((k for k, (i, j) in enumerate(cells) if i >= H or j >= W), len(cells))
        checked = cells[:k_oor]
        if len(checked) > _abi.MAX_FOOT:
            raise ValueError(f"the footprint has {len(checked)} cells; the kernels take at most {_abi.MAX_FOOT}")
        grid = max(8, -(-max(H, W) // 4) * 4)
        cfg = self.cfg.replace(grid=grid, n_beams=0, n_obst=0)
        c = _abi.make_cfg(cfg)
        c.n_foot = len(checked)
        for k, (i, j) in enumerate(checked):
            c.foot_di[k], c.foot_dj[k] = i - grid // 2, j - grid // 2  # the kernel reads grid/2 + offset = i
        # the lidar threshold: is_collision2 compares with the module constant ROBOT_RSIZE
        # (ffmp.py:112), not with self.robot_rsize (which only shapes the footprint above)
        c.robot_r = float(ROBOT_RSIZE)
        if len(self._cfg_cache) >= 64:
            self._cfg_cache.clear()
        complete = k_oor == len(cells)
        self._cfg_cache[key] = (c, self.robot_grids, complete, self.cfg)
        return c, complete

    @staticmethod
    def _map2d(local_map):
        """local_map_info as the 2-D plane the reference's [i, j] indexing reads: (H, W) or (H, W, 1);
        more channels make `local_map_info[i, j] > 0` an array whose truth value is ambiguous."""
        m = np.asarray(local_map)
        if m.ndim == 3:
            if m.shape[2] != 1:
                raise ValueError("The truth value of an array with more than one element is ambiguous "
                                 f"(local_map of shape {m.shape}: ffmp.py:101 tests local_map_info[i, j] > 0)")
            m = m[:, :, 0]
        if m.ndim != 2:
            raise ValueError(f"local_map must be (H,W) or (H,W,1), got {np.shape(local_map)}")
        return m

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # One call of the legacy surface = one host->device copy of every input packed into a pinned
    # staging buffer, one ffmp_reward_done launch, one device->host copy of every output, all in one
    # library call (include/ffmp.h ffmp_reward_done_packed).  Packed layout (bytes): outputs reward f64 @0, d0 f64 @8 (in/out), done / is_goal /
    # collide u8 @16..18; inputs rel_goal f64[2] @24, is_first / collide_in / goal_in u8 @40..42,
    # scan f64[L] @48, the local map f32[G*G] after it (16-aligned).
    def _staging(self, nbytes: int):
        st = self._stage
        if st is None or st[0].numel() < nbytes:
            cap = max(4096, 1 << (int(nbytes) - 1).bit_length())
            hin = torch.empty(cap, dtype=torch.uint8, pin_memory=True)
            st = self._stage = (hin, torch.empty(cap, dtype=torch.uint8, device=self.device), hin.numpy())
        return st

    # without a local map, ffmp_reward_done_packed's kernel-argument form (flag 8): no copies
    # (FFMP_SINGLE_ARGS=0: the copy form, an A/B knob)
    PACKED_ARGS = os.environ.get("FFMP_SINGLE_ARGS", "1") != "0"

    def _reward_done(self, rel_goal, is_first: bool, d0: float, scan=None, local_map=None,
                     collide_in=None, goal_in=None):
        lib = _abi.load()
        m = None
        shape = (self.cfg.grid, self.cfg.grid)
        if local_map is not None:
            m = self._map2d(local_map)
            shape = m.shape
        cfg_c, complete = self._legacy_cfg(shape)
        grid = cfg_c.grid
        # the scan as float64: None (the reference's list head, src/train.py:97) -> NaN, which like
        # None and 0.0 never counts as a hit (`bool(r) and r < 0.13`, ffmp.py:112: NaN < 0.13 is false)
        vals = None if scan is None else np.asarray(scan, dtype=np.float64).reshape(-1)
        L = 0 if vals is None else vals.size
        moff = -(-(48 + 8 * L) // 16) * 16
        nbytes = moff + (0 if m is None else 4 * grid * grid)
        hin, din, hnp = self._staging(nbytes)
        hnp[8:16].view(np.float64)[0] = d0
        hnp[24:40].view(np.float64)[:] = (float(rel_goal[0]), float(rel_goal[1]) if len(rel_goal) > 1 else 0.0)
        hnp[40:43] = (1 if is_first else 0, 1 if collide_in else 0, 1 if goal_in else 0)
        if L:
            hnp[48:48 + 8 * L].view(np.float64)[:] = vals
        if m is not None:
            plane = hnp[moff:nbytes].view(np.float32).reshape(grid, grid)
            if m.shape != (grid, grid):
                plane[:] = 0.0  # the padding (never read: every checked cell lies inside the map)
            plane[:m.shape[0], :m.shape[1]] = m
        flags = (0 if collide_in is None else 1) | (0 if goal_in is None else 2) | (0 if m is None else 4)
        if m is None and L <= _abi.PACKED_ARG_BEAMS and self.PACKED_ARGS:
            flags |= 8  # inputs as kernel arguments, outputs straight into the pinned block
        # one library call: the copy in, the kernel, the copy out, the stream synchronized
        _abi.check(lib.ffmp_reward_done_packed(C.byref(cfg_c), hin.data_ptr(), din.data_ptr(), nbytes, L, moff, grid,
                                               flags, C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)),
                   "ffmp_reward_done_packed")
        r, d0n = hnp[0:16].view(np.float64)
        if m is not None and not complete and not hnp[18]:
            # no occupied cell before the first one outside the map: the reference's loop reaches it
            raise IndexError(f"footprint cell outside the local map of shape {tuple(m.shape)} (ffmp.py:101)")
        return float(r), float(d0n), bool(hnp[16]), bool(hnp[17]), bool(hnp[18])

    # ---------------------------------------------------- reference methods
    def is_collision(self, local_map_info) -> bool:
        # the footprint test alone: one packed ffmp_reward_done call with the map and no scan
        return self._reward_done((1.0, 0.0), True, 0.0, local_map=local_map_info)[4]

    def is_collision2(self, scan_data) -> bool:
        vals = np.asarray(scan_data, dtype=np.float64).reshape(-1)  # None -> NaN: never a hit, as None
        if len(vals) == 0:
            return False
        # the lidar test alone (threshold ROBOT_RSIZE): one packed ffmp_reward_done call, no map
        hit = self._reward_done((1.0, 0.0), True, 0.0, scan=vals)[4]
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
