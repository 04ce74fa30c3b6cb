"""ORACLE — TEST INFRASTRUCTURE ONLY.  ctypes front end of oracle/ffmp_oracle.c.

`COracleVecEnv` has OracleVecEnv's constructor, attributes and reset / step / obs API, and is
bit-identical to it (tests/test_oracle_c.py); the stepping is compiled C, multi-threaded over
envs.  Used by tests/ as a checker at full grid sizes and by bench.py as the timed CPU baseline.
The product never imports this module (tests/test_host_abi.py::test_product_never_imports_oracle).

The library is built by `build()` below (called from __graft_entry__.build()): oracle/_build/
libffmp_oracle_v3.so (x86-64-v3: AVX2) and libffmp_oracle.so (baseline x86-64); `load()` picks
the v3 build when the host CPU has AVX2 / BMI2 / FMA / MOVBE / F16C.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional

import numpy as np

from .ffmp_oracle import F32, Cfg

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
SRC = os.path.join(HERE, "ffmp_oracle.c")
LIBS = {"v3": os.path.join(BUILD, "libffmp_oracle_v3.so"), "base": os.path.join(BUILD, "libffmp_oracle.so")}
# no fused multiply-adds, no fast-math, libm sin / cos / atan2 called one by one (as Python's math
# module does: no sincos fusion)
CFLAGS = ["-O3", "-std=c11", "-fPIC", "-shared", "-fopenmp", "-ffp-contract=off", "-fno-fast-math",
          "-fno-builtin-sin", "-fno-builtin-cos", "-fno-builtin-atan2"]
ARCH = {"v3": ["-march=x86-64-v3"], "base": ["-march=x86-64"]}

MAX_OBST, MAX_FOOT = 64, 128


def build(force: bool = False) -> None:
    """gcc the C oracle into oracle/_build (both ISA levels)."""
    os.makedirs(BUILD, exist_ok=True)
    for k, path in LIBS.items():
        if not force and os.path.exists(path) and os.path.getmtime(path) >= os.path.getmtime(SRC):
            continue
        tmp = path + ".tmp"
        subprocess.run(["gcc"] + CFLAGS + ARCH[k] + ["-o", tmp, SRC, "-lm"], check=True)
        os.replace(tmp, path)


def _host_has_v3() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    fl = set(line.split(":", 1)[1].split())
                    return {"avx2", "bmi2", "fma", "movbe", "f16c"} <= fl
    except OSError:
        pass
    return False


class _Cfg(C.Structure):
    _fields_ = ([(n, C.c_int32) for n in ("grid", "n_obst", "n_beams", "max_steps", "moving", "autoreset", "mode",
                                           "n_foot", "flow", "with_potential")] +
                [("foot_di", C.c_int32 * MAX_FOOT), ("foot_dj", C.c_int32 * MAX_FOOT)] +
                [(n, C.c_double) for n in ("res", "dt", "robot_r", "goal_thr", "W", "lidar_max", "goal_min",
                                            "goal_max", "obst_rmin", "obst_rmax", "obst_vmax", "start_clear",
                                            "goal_clear")] +
                [(n, C.c_float) for n in ("res_f", "half_f", "world_half_f", "half_ka_f", "half_kr_f", "rho0_f",
                                           "inv_rho0_f", "rho_min_f", "inv_2res_f", "pad_f")] +
                [("seed", C.c_uint64), ("beam_cs", C.c_void_p)])


_ENV_PTRS = ("pose", "goal", "d0", "obst", "obst_r", "t", "episode", "record", "term_record", "term_obs", "state_m",
             "potential", "flow", "state_g", "state_v", "state_t", "grad", "lidar", "reward", "done", "is_goal",
             "collision", "truncated")


class _Env(C.Structure):
    _fields_ = [("n", C.c_int64), ("env_offset", C.c_int64)] + [(n, C.c_void_p) for n in _ENV_PTRS]


_LIB = None


def load():
    global _LIB
    if _LIB is None:
        path = LIBS["v3"] if _host_has_v3() and os.path.exists(LIBS["v3"]) else LIBS["base"]
        if not os.path.exists(path):
            raise RuntimeError(f"C oracle not built ({path}); run __graft_entry__.build()")
        lib = C.CDLL(path)
        for name in ("ffmpo_reset", "ffmpo_step", "ffmpo_raster"):
            getattr(lib, name).restype = C.c_int
        lib.ffmpo_reset.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        lib.ffmpo_step.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
        lib.ffmpo_raster.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.path = path
        _LIB = lib
    return _LIB


class COracleVecEnv:
    """OracleVecEnv (oracle/ffmp_oracle.py) in compiled C; same arrays, same results."""

    def __init__(self, config, num_envs: int, env_offset: int = 0, with_potential: bool = True,
                 threads: Optional[int] = None):
        self.lib = load()
        cfg = self.cfg = Cfg.from_config(config)
        self.n, self.env_offset, self.with_potential = int(num_envs), int(env_offset), bool(with_potential)
        self.threads = int(threads) if threads else min(16, os.cpu_count() or 1)
        if cfg.n_obst > MAX_OBST or len(cfg.foot) > MAX_FOOT:
            raise ValueError("config exceeds the C oracle's limits")
        n, K, G, L = self.n, cfg.n_obst, cfg.grid, cfg.n_beams
        self.pose = np.zeros((n, 3)); self.goal = np.zeros((n, 2)); self.d0 = np.zeros(n)
        self.obst = np.zeros((n, K, 4)); self.obst_r = np.zeros((n, K))
        self.t = np.zeros(n, dtype=np.int32); self.episode = np.zeros(n, dtype=np.int32)
        self.record = np.zeros((n, 16 + 12 * K), dtype=F32)
        self.term_record = np.zeros_like(self.record)
        self.term_obs = np.zeros((n, 5), dtype=F32)
        self.state_m = np.zeros((n, 2, G, G), dtype=F32)
        self.potential = np.zeros((n, G, G), dtype=F32)
        self.flow = np.zeros((n, 2, G, G), dtype=F32) if cfg.flow else None
        self.state_g = np.zeros((n, 2), dtype=F32); self.state_v = np.zeros((n, 2), dtype=F32)
        self.state_t = np.zeros((n, 1), dtype=F32); self.grad = np.zeros((n, 2), dtype=F32)
        self.lidar = np.zeros((n, L), dtype=F32)
        self.reward = np.zeros(n, dtype=F32)
        self.done = np.zeros(n, dtype=bool); self.is_goal = np.zeros(n, dtype=bool)
        self.collision = np.zeros(n, dtype=bool); self.truncated = np.zeros(n, dtype=bool)
        self.err = 0
        self._beams = np.ascontiguousarray(cfg.beam_cs, dtype=np.float64)
        c = _Cfg(grid=G, n_obst=K, n_beams=L, max_steps=cfg.max_steps, moving=int(cfg.moving),
                 autoreset=int(cfg.autoreset), mode=cfg.mode, n_foot=len(cfg.foot), flow=int(cfg.flow),
                 with_potential=int(self.with_potential), res=cfg.res, dt=cfg.dt, robot_r=cfg.robot_r,
                 goal_thr=cfg.goal_thr, W=cfg.W, lidar_max=cfg.lidar_max, goal_min=cfg.goal_min,
                 goal_max=cfg.goal_max, obst_rmin=cfg.obst_rmin, obst_rmax=cfg.obst_rmax, obst_vmax=cfg.obst_vmax,
                 start_clear=cfg.start_clear, goal_clear=cfg.goal_clear, seed=cfg.seed & (2 ** 64 - 1),
                 beam_cs=self._beams.ctypes.data if L else None)
        for i, (di, dj) in enumerate(cfg.foot):
            c.foot_di[i], c.foot_dj[i] = di, dj
        for k in ("res_f", "half_f", "world_half_f", "half_ka_f", "half_kr_f", "rho0_f", "inv_rho0_f", "rho_min_f",
                  "inv_2res_f"):
            setattr(c, k, float(cfg.f[k]))
        self._c = c
        e = _Env(n=n, env_offset=self.env_offset)
        for name in _ENV_PTRS:
            a = getattr(self, name)
            if a is not None:
                assert a.flags["C_CONTIGUOUS"]
                setattr(e, name, a.ctypes.data)
        if not self.with_potential:
            e.potential = None
        self._e = e

    def reset(self, mask: Optional[np.ndarray] = None):
        if mask is None:
            rc = self.lib.ffmpo_reset(C.byref(self._c), C.byref(self._e), None, self.threads)
        else:
            m = np.ascontiguousarray(np.asarray(mask, dtype=bool).reshape(self.n)).view(np.uint8)
            rc = self.lib.ffmpo_reset(C.byref(self._c), C.byref(self._e), m.ctypes.data, self.threads)
        if rc < 0:
            raise RuntimeError("ffmpo_reset failed")
        return self.obs()

    def obs(self):
        d = {"state_m": self.state_m, "state_g": self.state_g, "state_v": self.state_v,
             "state_t": self.state_t, "grad": self.grad}
        if self.with_potential:
            d["potential"] = self.potential
        if self.cfg.n_beams:
            d["lidar"] = self.lidar
        if self.cfg.flow:
            d["flow"] = self.flow
        return d

    def step(self, actions):
        a = np.ascontiguousarray(np.asarray(actions, dtype=np.int64).reshape(self.n))
        rc = self.lib.ffmpo_step(C.byref(self._c), C.byref(self._e), a.ctypes.data, self.threads)
        if rc < 0:
            raise RuntimeError("ffmpo_step failed")
        self.err |= rc
        info = {"is_goal": self.is_goal, "collision": self.collision, "truncated": self.truncated,
                "step": self.t, "episode": self.episode}
        return self.obs(), self.reward, self.done, info
