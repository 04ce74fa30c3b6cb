"""FFMPVec — N batched FFMP environments resident in HBM, stepped by libffmp.

This is the new batched surface the north star asks for (the reference's
`FFMP` has no step()/reset(): src/gym_ffmp/envs/ffmp.py:77-83 is commented out
and src/train.py drives Gazebo over ROS instead, train.py:523-693).  One call of
`step(actions)` is one iteration of the reference main loop for every env:

    publish cmd_vel(commander(action))       train.py:668-673  -> unicycle integrator
    Gazebo / BEV nodes produce the next obs   train.py:116-165  -> raster + lidar kernels
    make_temporal_maps                        train.py:474-486  -> state_m [older, newest]
    rewarder2 / rewarder                      ffmp.py:167-188   -> collision, goal, reward, done
    step == MAX_STEPS -> done                 train.py:607-608  -> truncated
    done -> /episode_manager reset            train.py:611-664  -> auto-reset (Philox)

Observation tensors keep the consumer layout of train.py:44,543-557 with a
leading N: state_m (N,2,G,G) f32, state_g (N,2), state_v (N,2), state_t (N,1);
extras: potential (N,G,G), grad (N,2), lidar (N,L).

Every entry point goes through the HIP library; there is no CPU path.  The
returned obs dict holds the env's own device buffers (overwritten in place by
the next step/reset) unless `copy=True`.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple, Union

import torch

from . import _abi
from .config import PRESETS, FFMPConfig, beam_table, preset


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


class FFMPVec:
    """Batched FFMP env on one GPU.

    Args:
        num_envs: envs held by THIS process (a shard of the global batch).
        config: FFMPConfig or preset name ("C1".."C5").
        device: a cuda device (default: current).
        env_offset: global index of env 0 (shard start); RNG streams are keyed
            by the global index so trajectories do not depend on sharding.
        potential: also raster the potential plane (default True).
    """

    def __init__(self, num_envs: int, config: Union[FFMPConfig, str] = "C3",
                 device: Optional[Union[str, torch.device]] = None, env_offset: int = 0,
                 potential: bool = True, seed: Optional[int] = None):
        if isinstance(config, str):
            config = preset(config)
        if seed is not None:
            config = config.replace(seed=int(seed))
        self.cfg: FFMPConfig = config
        self.lib = _abi.load()
        if not torch.cuda.is_available():
            raise _abi.FFMPBackendError("FFMPVec needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if self.device.type != "cuda":
            raise ValueError(f"FFMPVec runs on a GPU device, got {self.device}")
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.num_envs = int(num_envs)
        if self.num_envs <= 0:
            raise ValueError("num_envs must be positive")
        self.env_offset = int(env_offset)
        self.with_potential = bool(potential)
        self._alloc()
        self._build_structs()
        self._needs_reset = True

    # ------------------------------------------------------------------ setup
    def _alloc(self):
        cfg, N, dev = self.cfg, self.num_envs, self.device
        G, K, L = cfg.grid, cfg.n_obst, cfg.n_beams
        f32, f64 = torch.float32, torch.float64
        e = lambda *s, dtype=f32: torch.empty(*s, dtype=dtype, device=dev)  # noqa: E731
        z = lambda *s, dtype=f32: torch.zeros(*s, dtype=dtype, device=dev)  # noqa: E731
        # state
        self.pose = z(N, 3, dtype=f64)
        self.goal = z(N, 2, dtype=f64)
        self.d0 = z(N, dtype=f64)
        self.obst = z(N, max(K, 1), 4, dtype=f64)
        self.obst_r = z(N, max(K, 1), dtype=f64)
        self.t = z(N, dtype=torch.int32)
        self.episode = z(N, dtype=torch.int32)
        self.record = z(N, cfg.record_len())
        self.err = z(1, dtype=torch.int32)
        # obs
        self.state_m = e(N, 2, G, G)
        self.state_g = z(N, 2)
        self.state_v = z(N, 2)
        self.state_t = z(N, 1)
        self.potential = e(N, G, G) if self.with_potential else None
        self.grad = z(N, 2)
        self.lidar = z(N, L) if L > 0 else None
        # outputs
        self.reward = z(N)
        self.done = z(N, dtype=torch.bool)
        self.is_goal = z(N, dtype=torch.bool)
        self.collision = z(N, dtype=torch.bool)
        self.truncated = z(N, dtype=torch.bool)
        # tables
        self.beam_cs = torch.as_tensor(beam_table(L), dtype=f64).to(dev) if L > 0 else None

    def _build_structs(self):
        self._cfg_c = _abi.make_cfg(self.cfg, _ptr(self.beam_cs) or 0)
        self._state_c = _abi.StateT(self.pose.data_ptr(), self.goal.data_ptr(), self.d0.data_ptr(),
                                    self.obst.data_ptr(), self.obst_r.data_ptr(), self.t.data_ptr(),
                                    self.episode.data_ptr(), self.record.data_ptr(), self.err.data_ptr())
        self._obs_c = _abi.ObsT(self.state_m.data_ptr(), self.state_g.data_ptr(), self.state_v.data_ptr(),
                                self.state_t.data_ptr(), _ptr(self.potential), self.grad.data_ptr(),
                                _ptr(self.lidar))
        self._out_c = _abi.OutT(self.reward.data_ptr(), self.done.data_ptr(), self.is_goal.data_ptr(),
                                self.collision.data_ptr(), self.truncated.data_ptr())

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # --------------------------------------------------------------- gym API
    @property
    def obs(self) -> Dict[str, torch.Tensor]:
        d = {"state_m": self.state_m, "state_g": self.state_g, "state_v": self.state_v, "state_t": self.state_t,
             "grad": self.grad}
        if self.potential is not None:
            d["potential"] = self.potential
        if self.lidar is not None:
            d["lidar"] = self.lidar
        return d

    def _obs_out(self, copy: bool):
        o = self.obs
        return {k: v.clone() for k, v in o.items()} if copy else o

    def reset(self, seed: Optional[int] = None, mask: Optional[torch.Tensor] = None, copy: bool = False):
        """Reset all envs (mask None: new episodes 0 from `seed`) or only masked ones."""
        with torch.cuda.device(self.device):
            if seed is not None:
                self.cfg = self.cfg.replace(seed=int(seed))
                self._cfg_c = _abi.make_cfg(self.cfg, _ptr(self.beam_cs) or 0)
            m = None
            if mask is not None:
                m = mask.to(device=self.device, dtype=torch.bool).contiguous().view(torch.uint8)
                if m.numel() != self.num_envs:
                    raise ValueError("mask must have num_envs elements")
            initial = 1 if (mask is None) else 0
            s = self._stream()
            _abi.check(self.lib.ffmp_reset(C.byref(self._cfg_c), self.num_envs, self.env_offset, _ptr(m), initial,
                                           C.byref(self._state_c), C.byref(self._obs_c), s), "ffmp_reset")
            _abi.check(self.lib.ffmp_raster(C.byref(self._cfg_c), self.num_envs, self.record.data_ptr(), _ptr(m),
                                            C.byref(self._obs_c), s), "ffmp_raster")
            self._mask_keepalive = m
        self._needs_reset = False
        return self._obs_out(copy)

    def _actions(self, actions) -> torch.Tensor:
        a = torch.as_tensor(actions)
        if a.device != self.device or a.dtype != torch.int64:
            a = a.to(device=self.device, dtype=torch.int64)
        a = a.reshape(-1)
        if a.numel() != self.num_envs:
            raise ValueError(f"expected {self.num_envs} actions, got {a.numel()}")
        return a.contiguous()

    def step_state(self, actions: torch.Tensor) -> None:
        """Kernel 1 of a step: dynamics, lidar, reward/done, auto-reset, record."""
        a = self._actions(actions)
        self._act_keepalive = a
        _abi.check(self.lib.ffmp_step_state(C.byref(self._cfg_c), self.num_envs, self.env_offset, a.data_ptr(),
                                            C.byref(self._state_c), C.byref(self._obs_c), C.byref(self._out_c),
                                            self._stream()), "ffmp_step_state")

    def raster(self, mask: Optional[torch.Tensor] = None) -> None:
        """Kernel 2 of a step: state_m frames and potential plane (the HBM-bound hot kernel)."""
        m = None if mask is None else mask.to(device=self.device, dtype=torch.bool).contiguous().view(torch.uint8)
        _abi.check(self.lib.ffmp_raster(C.byref(self._cfg_c), self.num_envs, self.record.data_ptr(), _ptr(m),
                                        C.byref(self._obs_c), self._stream()), "ffmp_raster")

    def step(self, actions, copy: bool = False) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor, dict]:
        """Advance every env one step. Returns (obs, reward f32[N], done bool[N], info)."""
        if self._needs_reset:
            raise RuntimeError("call reset() before step()")
        with torch.cuda.device(self.device):
            self.step_state(actions)
            self.raster()
        info = {"is_goal": self.is_goal, "collision": self.collision, "truncated": self.truncated,
                "step": self.t, "episode": self.episode}
        if copy:
            info = {k: v.clone() for k, v in info.items()}
            return self._obs_out(True), self.reward.clone(), self.done.clone(), info
        return self.obs, self.reward, self.done, info

    # ------------------------------------------------------------ utilities
    def check_errors(self) -> None:
        """Raise if any step saw an action id outside 0..27 (it was run as action 3)."""
        v = int(self.err.item())
        if v:
            self.err.zero_()
            raise ValueError(f"invalid action id(s) passed to FFMPVec.step (error bits {v:#x})")

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Checkpoint of the simulator state (obs are re-derivable by raster())."""
        return {"pose": self.pose.clone(), "goal": self.goal.clone(), "d0": self.d0.clone(),
                "obst": self.obst.clone(), "obst_r": self.obst_r.clone(), "t": self.t.clone(),
                "episode": self.episode.clone(), "record": self.record.clone(),
                "seed": torch.tensor(self.cfg.seed, dtype=torch.int64), }

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for k in ("pose", "goal", "d0", "obst", "obst_r", "t", "episode", "record"):
            getattr(self, k).copy_(sd[k])
        seed = int(sd["seed"])
        if seed != self.cfg.seed:
            self.cfg = self.cfg.replace(seed=seed)
            self._cfg_c = _abi.make_cfg(self.cfg, _ptr(self.beam_cs) or 0)
        self.raster()
        self._needs_reset = False

    def hbm_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in vars(self).values() if isinstance(t, torch.Tensor))

    def __repr__(self):
        c = self.cfg
        return (f"FFMPVec(num_envs={self.num_envs}, G={c.grid}, K={c.n_obst}, L={c.n_beams}, "
                f"moving={c.moving}, device={self.device}, env_offset={self.env_offset})")


__all__ = ["FFMPVec", "PRESETS"]
