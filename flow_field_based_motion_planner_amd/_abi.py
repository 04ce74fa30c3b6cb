"""ctypes binding of libffmp (include/ffmp.h).

The shared library is built in-tree (`__graft_entry__.build()` or `make`) to
flow_field_based_motion_planner_amd/lib/libffmp.so.  There is NO fallback: if
the library is missing every device entry point raises FFMPBackendError.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional

from .config import MAX_FOOT, FFMPConfig

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FFMP_LIB", os.path.join(_HERE, "lib", "libffmp.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ffmp.h")

ABI_VERSION = 8
OBS_F32, OBS_U8F16 = 0, 1  # include/ffmp.h FFMP_OBS_*
MAX_SERIES = 16  # FFMP_MAX_SERIES (ffmp_temporal_maps)
PACKED_ARG_BEAMS = 360  # FFMP_PACKED_ARG_BEAMS (ffmp_reward_done_packed flag 8)


class FFMPBackendError(RuntimeError):
    """libffmp is missing, unloadable or returned an error."""


class CfgT(C.Structure):
    _fields_ = [
        ("grid", C.c_int32), ("n_obst", C.c_int32), ("n_beams", C.c_int32), ("max_steps", C.c_int32),
        ("moving", C.c_int32), ("autoreset", C.c_int32), ("collide_mode", C.c_int32), ("n_foot", C.c_int32),
        ("flow", C.c_int32), ("reserved0", C.c_int32),
        ("foot_di", C.c_int32 * MAX_FOOT), ("foot_dj", C.c_int32 * MAX_FOOT),
        ("res", C.c_double), ("dt", C.c_double), ("robot_r", C.c_double), ("goal_thr", C.c_double),
        ("world_half", C.c_double), ("lidar_max", C.c_double), ("goal_min", C.c_double), ("goal_max", C.c_double),
        ("obst_rmin", C.c_double), ("obst_rmax", C.c_double), ("obst_vmax", C.c_double),
        ("start_clear", C.c_double), ("goal_clear", C.c_double),
        ("res_f", C.c_float), ("half_f", C.c_float), ("world_half_f", C.c_float), ("half_ka_f", C.c_float),
        ("half_kr_f", C.c_float), ("rho0_f", C.c_float), ("inv_rho0_f", C.c_float), ("rho_min_f", C.c_float),
        ("inv_2res_f", C.c_float), ("cull_margin_f", C.c_float),
        ("seed", C.c_uint64), ("beam_cs", C.c_void_p),
    ]


class StateT(C.Structure):
    _fields_ = [("pose", C.c_void_p), ("goal", C.c_void_p), ("d0", C.c_void_p), ("obst", C.c_void_p),
                ("obst_r", C.c_void_p), ("t", C.c_void_p), ("episode", C.c_void_p), ("record", C.c_void_p),
                ("err", C.c_void_p), ("term_record", C.c_void_p), ("term_obs", C.c_void_p)]


class ObsT(C.Structure):
    _fields_ = [("state_m", C.c_void_p), ("state_g", C.c_void_p), ("state_v", C.c_void_p),
                ("state_t", C.c_void_p), ("potential", C.c_void_p), ("grad", C.c_void_p), ("lidar", C.c_void_p),
                ("flow", C.c_void_p), ("state_m_stride", C.c_int64), ("state_m_frame_stride", C.c_int64),
                ("format", C.c_int32), ("reserved", C.c_int32)]


class OutT(C.Structure):
    _fields_ = [("reward", C.c_void_p), ("done", C.c_void_p), ("is_goal", C.c_void_p),
                ("collide", C.c_void_p), ("truncated", C.c_void_p)]


class EpisodeT(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("reach_bits", "reach_len", "reach_rate", "step", "episode",
                                          "total_step", "is_first", "complete", "totals")]


EP_TOTALS = 8
EP_ARMED, EP_RESET_ITER = 1, 2


def make_cfg(cfg: FFMPConfig, beam_cs_ptr: int = 0) -> CfgT:
    c = CfgT()
    c.grid, c.n_obst, c.n_beams, c.max_steps = cfg.grid, cfg.n_obst, cfg.n_beams, cfg.max_steps
    c.moving, c.autoreset, c.collide_mode = int(cfg.moving), int(cfg.autoreset), cfg.mode
    c.flow = int(bool(cfg.flow))
    fp = cfg.footprint
    c.n_foot = len(fp)
    for k, (di, dj) in enumerate(fp):
        c.foot_di[k], c.foot_dj[k] = di, dj
    c.res, c.dt, c.robot_r, c.goal_thr = cfg.res, cfg.dt, cfg.robot_r, cfg.goal_thr
    c.world_half, c.lidar_max, c.goal_min, c.goal_max = cfg.W, cfg.lidar_range, cfg.goal_min, cfg.goal_hi
    c.obst_rmin, c.obst_rmax, c.obst_vmax = cfg.obst_rmin, cfg.obst_rmax, cfg.obst_vmax
    c.start_clear, c.goal_clear = cfg.start_clear, cfg.goal_clear
    for k, v in cfg.f32_constants().items():
        setattr(c, k, float(v))  # float32 values are exact in the c_float field
    c.seed = int(cfg.seed)
    c.beam_cs = beam_cs_ptr or None
    return c


_P = C.c_void_p
_I64 = C.c_int64
_I32 = C.c_int32
_SIGS = {
    "ffmp_abi_version": (C.c_int, []),
    "ffmp_last_error": (C.c_char_p, []),
    "ffmp_layout": (_I64, [_I32]),
    "ffmp_set_tuning": (_I32, [_I32, _I32]),
    "ffmp_footprint": (C.c_int, [_I32, C.c_double, C.c_double, _P, _P, _I32]),
    "ffmp_reset": (C.c_int, [C.POINTER(CfgT), _I64, _I64, _P, _I32, C.POINTER(StateT), C.POINTER(ObsT), _P]),
    "ffmp_step_state": (C.c_int, [C.POINTER(CfgT), _I64, _I64, _P, C.POINTER(StateT), C.POINTER(ObsT),
                                  C.POINTER(OutT), _P]),
    "ffmp_raster": (C.c_int, [C.POINTER(CfgT), _I64, _P, _P, C.POINTER(ObsT), _P]),
    "ffmp_raster_ex": (C.c_int, [C.POINTER(CfgT), _I64, _P, _P, C.POINTER(ObsT), _I32, _I32, _P]),
    "ffmp_step": (C.c_int, [C.POINTER(CfgT), _I64, _I64, _P, C.POINTER(StateT), C.POINTER(ObsT),
                            C.POINTER(OutT), _P]),
    "ffmp_step_fused": (C.c_int, [C.POINTER(CfgT), _I64, _I64, _P, C.POINTER(StateT), C.POINTER(ObsT),
                                  C.POINTER(OutT), _I32, _P]),
    "ffmp_step_skewed": (C.c_int, [C.POINTER(CfgT), _I64, _I64, _P, C.POINTER(StateT), C.POINTER(ObsT),
                                   C.POINTER(OutT), _P, _I32, _I32, _P]),
    "ffmp_step_skewed_check": (C.c_int, [C.POINTER(CfgT), _I32, _I32]),
    "ffmp_policy_reactive": (C.c_int, [C.POINTER(CfgT), _I64, C.POINTER(ObsT), _P, _P]),
    "ffmp_reward_done": (C.c_int, [C.POINTER(CfgT), _I64, _P, _I32, _P, _I64, _P, _P, _P, _P, _P, _P, _P, _P,
                                   _P, _P]),
    "ffmp_footprint_collision": (C.c_int, [C.POINTER(CfgT), _I64, _P, _I64, _P, _P]),
    "ffmp_scan_collision": (C.c_int, [_I64, _I32, _P, C.c_double, _P, _P, _P]),
    "ffmp_scan_collision_f64": (C.c_int, [_I64, _I32, _P, C.c_double, _P, _P, _P]),
    "ffmp_check_exact_math": (C.c_int, [_I32, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "ffmp_conv2d_fwd_bf16": (C.c_int, [_P, _P, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32,
                                       _P]),
    "ffmp_conv2d_wgrad_bf16": (C.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    "ffmp_reward_done_packed": (C.c_int, [C.POINTER(CfgT), _P, _P, _I64, _I32, _I64, _I32, _I32, _P]),
    "ffmp_conv2d_dgrad_bf16": (C.c_int, [_P, _P, _P, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _I32, _P]),
    "ffmp_conv2d_check": (C.c_int, [_I32] * 10),
    "ffmp_episode_init": (C.c_int, [_I64, _P, _I32, C.POINTER(EpisodeT), _P]),
    "ffmp_episode_update": (C.c_int, [_I64, C.POINTER(OutT), _I32, _I32, C.c_double, _I32, C.POINTER(EpisodeT),
                                      _P]),
    "ffmp_temporal_maps": (C.c_int, [_I64, _P, C.POINTER(_I64), _I32, _I64, _I64, _I32, _P, _P, _P]),
    "ffmp_bev_image": (C.c_int, [_I64, _I32, _P, _I64, _P, _I64, C.c_float, _P, _I64, _P]),
    "ffmp_ring_create": (C.c_int, [_I32, _I64, _I32, _P, _I64, C.POINTER(_P), C.POINTER(_P), C.POINTER(_I64)]),
    "ffmp_ring_info": (C.c_int, [_P, C.POINTER(C.c_double), _I32]),
    "ffmp_ring_rebuild": (C.c_int, [_P, C.c_uint64, _P, _I64, C.POINTER(_P), C.POINTER(_P), C.POINTER(_I64)]),
    "ffmp_ring_destroy": (C.c_int, [_P]),
    "ffmp_ring_pool_bytes": (_I64, [_I32]),
    "ffmp_ring_va_reserved": (_I64, [_I32]),
    "ffmp_ring_pool_trim": (C.c_int, [_I32, _I64, C.POINTER(_I64)]),
    "ffmp_ring_pair_forget": (C.c_int, [_I32, _P]),
    "ffmp_ring_pair_refs": (C.c_int, [_I32]),
    "ffmp_dlpack": (_P, [_P, _I32, _I32, _I32, C.POINTER(_I64), C.POINTER(_I64), _I32, _P]),
}

_LIB: Optional[C.CDLL] = None


def _hip_runtimes_mapped():
    """Distinct libamdhip64 files mapped into this process (Linux /proc/self/maps)."""
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})
    except OSError:  # pragma: no cover
        return []


def load(path: Optional[str] = None) -> C.CDLL:
    """Load libffmp once; raise FFMPBackendError if it is missing.

    torch (ROCm wheel) ships its own libamdhip64 with the same soname as
    /opt/rocm's.  Importing torch FIRST makes libffmp's libamdhip64.so.7 resolve
    to torch's copy, so the process holds ONE HIP runtime (two runtimes in one
    process cannot both open the GPU)."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    try:
        import torch  # noqa: F401  (binds libamdhip64.so.7 to torch's runtime)
    except ImportError:  # pragma: no cover - pure C users
        pass
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FFMPBackendError(
            f"libffmp not built: {p} is missing (run `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make` at the repo root). There is no CPU fallback.")
    try:
        lib = C.CDLL(p)
    except OSError as exc:  # pragma: no cover - environment specific
        raise FFMPBackendError(f"cannot load {p}: {exc}") from exc
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    rts = _hip_runtimes_mapped()
    if len(rts) > 1:
        raise FFMPBackendError(f"two HIP runtimes are loaded in this process: {rts}; import torch before "
                               "loading libffmp (flow_field_based_motion_planner_amd._abi.load does this)")
    if lib.ffmp_abi_version() != ABI_VERSION:
        raise FFMPBackendError(f"libffmp ABI {lib.ffmp_abi_version()} != expected {ABI_VERSION}")
    if path is None:
        _LIB = lib
    return lib


def check(rc: int, what: str = "libffmp") -> None:
    if rc != 0:
        msg = load().ffmp_last_error().decode(errors="replace")
        raise FFMPBackendError(f"{what} failed (rc={rc}): {msg}")


def verify_layout(lib: Optional[C.CDLL] = None) -> None:
    """Compare ctypes struct layouts with the compiled library's."""
    lib = lib or load()
    want = {
        0: C.sizeof(CfgT), 1: C.sizeof(StateT), 2: C.sizeof(ObsT), 3: C.sizeof(OutT),
        4: CfgT.res.offset, 5: CfgT.res_f.offset, 6: CfgT.seed.offset, 7: CfgT.beam_cs.offset,
        8: C.sizeof(EpisodeT),
        9: ObsT.format.offset,
    }
    for k, v in want.items():
        got = lib.ffmp_layout(k)
        if got != v:
            raise FFMPBackendError(f"ABI layout mismatch (item {k}): library {got}, ctypes {v}")


TUNE_RASTER_CPB, TUNE_RASTER_NT, TUNE_RASTER_XCD, TUNE_ENV_WAVES, TUNE_ENV_LANES, TUNE_RING_EXTRA = 1, 2, 3, 4, 5, 6
TUNE_CONV_MFMA, TUNE_CONV_KYS, TUNE_CONV_LB, TUNE_CONV_WGPF, TUNE_CONV_BA2, TUNE_CONV_MBW, TUNE_CONV_PLANAR = (
    7, 8, 9, 10, 11, 12, 13)
TUNE_CONV_PIN, TUNE_CONV_WGDMA = 14, 15
RASTER_NT, RASTER_PLAIN, RASTER_XCD, RASTER_NEWEST = 1, 2, 4, 8
RASTER_TILE2, RASTER_TILE4, RASTER_TILE8 = 16, 32, 64
RASTER_NARROW = 128  # FFMP_OBS_U8F16: 4 cells per lane instead of 16
RASTER_TILE16 = 256
RASTER_MID8 = 512  # FFMP_OBS_U8F16: 8 cells per lane


def set_tuning(key: int, value: int) -> int:
    """Process-wide launch-shape tuning (include/ffmp.h FFMP_TUNE_*); returns the previous value."""
    prev = load().ffmp_set_tuning(int(key), int(value))
    if prev < 0:
        check(prev, "ffmp_set_tuning")
    return prev


def ring_pool_trim(device: int, keep_bytes: int = 0) -> int:
    """Give back the physical memory of the frame-ring pieces parked in the process pool of
    `device` beyond keep_bytes (include/ffmp.h ffmp_ring_pool_trim; the addresses stay reserved).
    Returns the bytes released."""
    out = C.c_int64(0)
    check(load().ffmp_ring_pool_trim(int(device), int(keep_bytes), C.byref(out)), "ffmp_ring_pool_trim")
    return int(out.value)


def ring_pair_forget(device: int, partner: Optional[int] = None) -> int:
    """Forget the ring-pairing references kept for the partner plane at address `partner` (None:
    all of `device`'s), e.g. when the plane is freed (include/ffmp.h ffmp_ring_pair_forget)."""
    rc = load().ffmp_ring_pair_forget(int(device), partner)
    if rc < 0:
        check(rc, "ffmp_ring_pair_forget")
    return rc


# ----------------------------------------------------------------- DLPack (device memory -> torch)
# torch has no Python from_blob; libffmp builds a DLPack DLManagedTensor (with a C deleter, so
# nothing calls back into Python when torch frees it) and the capsule hands it to torch.
DL_CPU, DL_ROCM = 1, 10


def tensor_from_pointer(ptr: int, shape, strides, device_type: int = DL_ROCM, device_id: int = 0,
                        bits: int = 32, owner: Optional[int] = None):
    """A torch float tensor over existing memory `ptr` (element strides).  `owner`: a ring
    handle whose memory it is; the ring lives until its creator released it and every tensor
    made from it (and every view of those) is freed."""
    import torch.utils.dlpack as dl
    lib = load()
    nd = len(shape)
    shp = (C.c_int64 * nd)(*[int(s) for s in shape])
    std = (C.c_int64 * nd)(*[int(s) for s in strides])
    mt = lib.ffmp_dlpack(C.c_void_p(int(ptr)), device_type, device_id, nd, shp, std, bits, owner)
    if not mt:
        check(-1, "ffmp_dlpack")
    new_capsule = C.pythonapi.PyCapsule_New
    new_capsule.restype = C.py_object
    new_capsule.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p]
    return dl.from_dlpack(new_capsule(mt, b"dltensor", None))


class SeamlessRing:
    """`slots` frame planes of `plane_shape` in device memory plus a virtual slot `slots` that is
    a second mapping of slot 0 (include/ffmp.h ffmp_ring_create), handed to torch as ONE tensor
    (slots + 1, *plane) with the slot stride.  `partner`: the tensor the raster writes in
    lockstep with each slot (the potential plane; its contents are overwritten) — slot pieces
    are chosen to pair well with it.  The ring's pieces return to the process pool when its
    tensor and every view of it are freed (and the SeamlessRing object is gone)."""

    def __init__(self, device_id: int, plane_shape, slots: int, bits: int = 32, partner=None):
        self.lib = load()
        self.device_id, self.plane_shape, self.slots, self.bits = int(device_id), tuple(plane_shape), int(slots), bits
        slot_bytes = bits // 8
        for d in plane_shape:
            slot_bytes *= int(d)
        ring, base, stride = _P(), _P(), _I64()
        pp, pb = self._partner(partner)
        check(self.lib.ffmp_ring_create(self.device_id, int(slot_bytes), self.slots, pp, pb, C.byref(ring),
                                        C.byref(base), C.byref(stride)), "ffmp_ring_create")
        self.handle = None
        self.tensor = None
        self.rebuilds = 0
        self.reverts = 0
        self._prev = None  # (handle, tensor, slot_stride) of the ring before an undecided rebuild
        self._adopt(ring, base, stride)

    @staticmethod
    def _partner(partner):
        if partner is None:
            return None, 0
        return partner.data_ptr(), partner.numel() * partner.element_size()

    def _adopt(self, ring, base, stride, zero: bool = True, keep_old: bool = False) -> None:
        """Wrap a fresh ring as the (slots + 1, *plane) tensor (zeroed unless `zero` is False);
        this object keeps the creator's reference (the handle) so the ring can be rebuilt.
        keep_old: the previous ring stays alive (revert() / drop_previous())."""
        esize = self.bits // 8
        try:
            inner = [1]
            for d in reversed(self.plane_shape[1:]):
                inner.insert(0, inner[0] * int(d))
            shape = (self.slots + 1,) + self.plane_shape
            strides = (stride.value // esize,) + tuple(inner)
            t = tensor_from_pointer(base.value, shape, strides, DL_ROCM, self.device_id, self.bits, owner=ring.value)
            if zero:
                t[:self.slots].zero_()  # stream-ordered with the launches that follow
        except Exception:
            self.lib.ffmp_ring_destroy(ring)
            raise
        self.drop_previous()
        old = (self.handle, self.tensor, getattr(self, "slot_stride", None))
        self.handle, self.tensor, self.slot_stride = ring.value, t, stride.value
        if keep_old:
            self._prev = old
        elif old[0] is not None:
            self.lib.ffmp_ring_destroy(C.c_void_p(old[0]))

    def rebuild(self, slot_mask: int, partner=None, keep_old: bool = False) -> None:
        """Replace the pieces of the slots in slot_mask (ffmp_ring_rebuild); `tensor` becomes a new
        tensor — views of the old one must not be used any more.  Kept slots keep their bytes
        (the same memory as the old ring's), replaced ones are undefined.  keep_old: the old ring
        stays alive until drop_previous() (keep the new one) or revert() (back to the old one),
        so that a caller can time both."""
        ring, base, stride = _P(), _P(), _I64()
        pp, pb = self._partner(partner)
        check(self.lib.ffmp_ring_rebuild(C.c_void_p(self.handle), int(slot_mask), pp, pb, C.byref(ring),
                                         C.byref(base), C.byref(stride)), "ffmp_ring_rebuild")
        self.rebuilds += 1
        self._adopt(ring, base, stride, zero=False, keep_old=keep_old)

    def drop_previous(self) -> None:
        """Keep the current ring: release the one an undecided rebuild(keep_old=True) replaced."""
        prev, self._prev = self._prev, None
        if prev is not None:
            self.lib.ffmp_ring_destroy(C.c_void_p(prev[0]))

    def revert(self) -> None:
        """Undo the last rebuild(keep_old=True): the previous ring (and its tensor) is current
        again; the rebuilt one is released (its new pieces return to the pool once every view of
        its tensor is gone)."""
        if self._prev is None:
            raise RuntimeError("SeamlessRing.revert: no rebuild to undo")
        cur = self.handle
        self.handle, self.tensor, self.slot_stride = self._prev
        self._prev = None
        self.reverts += 1
        self.lib.ffmp_ring_destroy(C.c_void_p(cur))

    def info(self) -> dict:
        out = (C.c_double * 6)()
        self.lib.ffmp_ring_info(C.c_void_p(self.handle), out, 6)
        return {"pieces": int(out[0]), "pieces_new": int(out[1]), "pair_probes": int(out[2]),
                "pair_gbs_min": round(out[3], 1), "pair_gbs_max": round(out[4], 1), "pair_scale": int(out[5]),
                "rebuilds": self.rebuilds, "reverts": self.reverts}

    def __del__(self):
        try:
            self.drop_previous()
            if self.handle is not None:
                self.lib.ffmp_ring_destroy(C.c_void_p(self.handle))
                self.handle = None
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def footprint_from_lib(grid: int, res: float, robot_r: float):
    lib = load()
    di = (C.c_int32 * MAX_FOOT)()
    dj = (C.c_int32 * MAX_FOOT)()
    n = lib.ffmp_footprint(grid, res, robot_r, C.cast(di, _P), C.cast(dj, _P), MAX_FOOT)
    if n < 0:
        check(n, "ffmp_footprint")
    return [(di[k], dj[k]) for k in range(min(n, MAX_FOOT))]
