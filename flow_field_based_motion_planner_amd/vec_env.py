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
the next step/reset) unless `copy=True`.  With a frame ring (frame_window > 2)
`state_m` is a view of the current pair of ring slots, so take it from each
step's return value (or `env.state_m`) rather than keeping the first one.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Dict, Optional, Tuple, Union

import numpy as np
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
        keep_terminal: also keep every env's post-step state before auto-reset
            (`term_record` (N, record_len) and `term_obs` (N, 5) = state_g, state_v, state_t):
            what a transition store needs for envs that just finished (ReplayMemory).
        frame_window: W >= 2 frames per env kept in HBM.  W > 2: a slot-major ring `frames`
            (W, N, G, G) and `state_m` = the (N,2,G,G) view frames[p:p+2].transpose(0, 1) of the
            current [older, newest] pair.  Each step slides the pair by one slot and writes only
            the new frame (plus the older one of envs that reset): the temporal stack of
            make_temporal_maps (train.py:474-486) kept in place instead of re-written, as one
            contiguous plane per slot.  Every W-1 steps the pair wraps to slot 0 (both frames
            written).  W = 2: the contiguous (N,2,G,G) layout, both frames written every step.
            None: 8 for large batches when HBM allows, else 2.
        seamless: W > 2 only.  True: the ring is HIP virtual memory with one extra virtual slot
            mapped onto slot 0's pages (include/ffmp.h ffmp_ring_create), so the pair never
            wraps and every step writes only the new frame; `frames` is (W+1, N, G, G) with
            frames[W] aliasing frames[0].  None (default): seamless when the device supports
            it, else the wrapping ring.  False: always the wrapping ring.
        fused: True: every step is ONE launch (ffmp_step_fused: one block per env steps the env,
            then rasters its plane); False: the env kernel, then the raster; None (default): the
            autotune times both on this instance and keeps the faster (small batches: False).
        tuning: a previous instance's `tuning()` (launch shapes, one- or two-launch step): used
            instead of the autotune (e.g. for profiling runs that should contain only timed
            launches); the seamless ring's slot repair still runs.
        hbm_budget: bytes of HBM this instance may hold, at steady state and while it is built
            (autotune placement tries and the ring's pairing candidates included): caps the frame
            window W, the ring's extra pairing pieces (FFMP_TUNE_RING_EXTRA) and the relocation /
            placement retries (each holds another arena + a spacer).  None: W and the retries are
            sized from free HBM (60 % for the ring).  Pieces a closed instance's ring left in the
            process pool are reused by later rings and are not charged to this one.  `hbm_bytes()`
            / `hbm_peak_bytes` report what it holds / held at most.
        obs_format: "f32" (default): the reference consumer layout, state_m float32 0/255
            (train.py:543-545) and a float32 potential plane.  "u8f16": the compact layout
            (include/ffmp.h FFMP_OBS_U8F16) for consumers that convert on load — state_m uint8
            with the same 0/255 values (`state_m.float()` is the f32 layout bit for bit) and the
            potential plane as float16 (the float32 value rounded to nearest even): 3 instead of
            8 bytes per cell of a step's raster.  With cfg.flow the flow planes are float16 too.
        bev_series: k > 0 (needs cfg.flow): also keep the last k 4-channel BEV images [occupancy,
            R, G, B] of every env (ffmp_bev_image: the newest frame and its motion flow as colour),
            a ring `bev` (k, N, 4, G, G) written after every step / reset; bev_maps() is the input of
            the reference's 12-channel option (train.py:66: "(occupancy(MONO) + flow(RGB)) *
            series(3 steps)", k = 3).  One extra elementwise launch per step.
        info_format: "dict" (default): step()'s info is one dict of (N,) device tensors (is_goal,
            collision, truncated, step, episode).  "list": gym 0.17/0.18 VectorEnv's form, a tuple
            of N per-env dicts of Python scalars (one device -> host copy per step).
    """

    def __init__(self, num_envs: int, config: Union[FFMPConfig, str] = "C3",
                 device: Optional[Union[str, torch.device]] = None, env_offset: int = 0,
                 potential: bool = True, seed: Optional[int] = None, arena: bool = True,
                 autotune: bool = True, pipeline: Optional[int] = None, keep_terminal: bool = False,
                 frame_window: Optional[int] = None, seamless: Optional[bool] = None,
                 fused: Optional[bool] = None, tuning: Optional[dict] = None, obs_format: str = "f32",
                 hbm_budget: Optional[int] = None, bev_series: int = 0, info_format: str = "dict"):
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
        if obs_format not in self.OBS_FORMATS:
            raise ValueError(f"obs_format must be one of {sorted(self.OBS_FORMATS)}, got {obs_format!r}")
        self.obs_format = obs_format
        if info_format not in self.INFO_FORMATS:
            raise ValueError(f"info_format must be one of {self.INFO_FORMATS}, got {info_format!r}")
        self.info_format = info_format
        self._fmt, self._frame_dtype, self._pot_dtype = self.OBS_FORMATS[obs_format]
        self._fes = torch.empty((), dtype=self._frame_dtype).element_size()  # bytes per frame cell
        self._pes = torch.empty((), dtype=self._pot_dtype).element_size()    # bytes per potential cell
        self.env_offset = int(env_offset)
        self.with_potential = bool(potential)
        self.hbm_budget = None if hbm_budget is None else int(hbm_budget)
        self.hbm_peak_bytes = 0
        self.arena = bool(arena)
        self.keep_terminal = bool(keep_terminal)
        self.placement = None
        self.raster_shape = (0, 0)  # (cells per block, FFMP_RASTER_* flags); 0, 0 = library default
        self.raster_shape_newest = (0, 0)  # the same for newest-only launches (frame ring)
        # the BEV image ring (bev_series) is an arena buffer like the planes: counted by the HBM
        # budget, the auto frame window and the ring's pairing spare
        self.bev_series = int(bev_series)
        if self.bev_series:
            if not self.cfg.flow:
                raise ValueError("bev_series needs FFMPConfig(flow=True) (the flow planes it colours)")
            if not 1 <= self.bev_series <= _abi.MAX_SERIES:
                raise ValueError(f"bev_series must be in [1, {_abi.MAX_SERIES}]")
        self.frame_window = self._pick_window(frame_window)
        self._seamless_req = seamless if self.frame_window > 2 else False
        if seamless and self.frame_window == 2:
            raise ValueError("seamless=True needs frame_window > 2")
        self.ring = "contiguous" if self.frame_window == 2 else "wrap"  # or "seamless" (set by _alloc)
        self.ring_meta = None
        self.fused = bool(fused) if fused is not None else False  # autotune may switch it on
        self._fused_req = fused
        self.fused_flags = _abi.RASTER_NT
        self._wpos = 0  # frame slot of state_m[:, 0]
        # temporal_maps(k): physical ring slots of the newest frames, newest first (lag 0, 1, ...),
        # and whether every env's lags beyond them are clamped away (a full reset) or unknown
        # (a checkpoint reload re-rasters only the [older, newest] pair)
        self._hist = []
        self._hist_from_reset = False
        self._alloc()
        self._bev_pos = 0       # ring slot of the newest image
        self._bev_hist = []     # slots of the newest images, newest first (as _hist)
        self._bev_from_reset = False
        G2 = self.cfg.grid * self.cfg.grid
        if pipeline is None:
            pipeline = 1  # measured: no net gain on MI355X (profiles/r01_pipeline.txt, r03b_pipeline.txt)
        self.pipeline_slices = max(1, min(int(pipeline), self.num_envs))
        if self.pipeline_slices > 1 and fused:
            raise ValueError("pipeline > 1 and fused=True are exclusive")
        if self.pipeline_slices > 1:
            self._fused_req = False
        plane_bytes = self.num_envs * G2 * (2 * self._fes + (self._pes if potential else 0) +
                                            (2 * self._pes if self.cfg.flow else 0))
        paired = self.ring == "seamless" and self.with_potential
        if paired and plane_bytes >= self.RELOCATE_MIN_BYTES and (tuning is not None or autotune):
            self._relocate_partner(self.PARTNER_TRIES if plane_bytes >= self.REPLACE_MIN_BYTES
                                   else self.PARTNER_TRIES_SMALL)
        self._build_structs()
        if tuning is not None:
            self._apply_tuning(tuning)
            if paired and plane_bytes >= self.RELOCATE_MIN_BYTES:
                self._repair_slots()
                self.placement = dict(self.placement, ring=self.ring_meta)
        elif autotune and plane_bytes >= self.AUTOTUNE_MIN_BYTES:
            self._autotune_raster()
            # the seamless ring already paired its slots with the potential plane; a new arena
            # would undo that
            if self.arena and plane_bytes >= self.REPLACE_MIN_BYTES and not paired:
                self._retry_placement()
            if paired and plane_bytes >= self.RELOCATE_MIN_BYTES:
                self._repair_slots()
                self._recheck_fused()
            if self.placement is not None and self.ring_meta is not None:
                self.placement = dict(self.placement, ring=self.ring_meta)
        self.pool_released_bytes = 0
        if self.ring == "seamless":
            # the pairing references of the planes this instance paired against and then dropped
            # (relocation tries): those planes are freed, a later plane may take their address
            self._forget_partners(keep=self.potential)
        if self.release_pool and self.ring == "seamless":
            # the pairing candidates this instance did not choose, the rings its relocation /
            # repair dropped: their memory goes back to the device (addresses stay reserved)
            torch.cuda.synchronize(self.device)
            self.pool_released_bytes = _abi.ring_pool_trim(self.device.index, self.pool_keep_bytes)
            if self.ring_meta is not None:
                self.ring_meta = dict(self.ring_meta, pool_released_bytes=self.pool_released_bytes)
                if self.placement is not None and "ring" in self.placement:
                    self.placement = dict(self.placement, ring=self.ring_meta)
        self._needs_reset = True

    # ------------------------------------------------------------------ setup
    # After construction (and on close) the frame-ring pieces parked in the process pool — pairing
    # candidates not chosen, rings dropped by the relocation / slot repair — are released
    # (ffmp_ring_pool_trim): at C3 they were ~65 GB beside the instance's 77 GB (round 3).  A
    # process that builds envs in a loop may keep a floor of pieces for the next one (reused first).
    release_pool = True
    pool_keep_bytes = 0
    _pair_partners = ()  # potential-plane addresses this instance's rings were paired against

    @staticmethod
    def _forget_at_exit(device: int, box: list) -> None:
        """weakref.finalize of an instance dropped without close(): its planes' pairing references
        go with it (a later instance whose plane lands at the same address — torch's caching
        allocator hands it out again — must not be judged against another plane's probe)."""
        for ptr in box:
            _abi.ring_pair_forget(device, ptr)
        box.clear()

    def _note_partner(self) -> None:
        if self.potential is not None:
            self._pair_partners = tuple(set(self._pair_partners) | {self.potential.data_ptr()})
            box = getattr(self, "_partner_box", None)
            if box is None:
                import weakref
                box = self._partner_box = []
                weakref.finalize(self, FFMPVec._forget_at_exit, self.device.index, box)
            box[:] = list(self._pair_partners)

    def _forget_partners(self, keep: Optional[torch.Tensor] = None) -> None:
        """Forget the ring-pairing references of the partner planes this instance no longer holds
        (trimming the pool had erased every instance's)."""
        k = None if keep is None else keep.data_ptr()
        for ptr in self._pair_partners:
            if ptr != k:
                _abi.ring_pair_forget(self.device.index, ptr)
        self._pair_partners = () if k is None else (k,)
        box = getattr(self, "_partner_box", None)
        if box is not None:
            box[:] = list(self._pair_partners)

    OBS_FORMATS = {"f32": (_abi.OBS_F32, torch.float32, torch.float32),
                   "u8f16": (_abi.OBS_U8F16, torch.uint8, torch.float16)}
    _ARENA_ALIGN = 2 << 20
    WINDOW_DEFAULT = 8
    WINDOW_HBM_FRACTION = 0.6  # auto window: frames + other planes within this share of free HBM

    def _arena_estimate(self, with_frames: bool) -> int:
        """Bytes of the arena _alloc carves (2 MiB-aligned buffers)."""
        off = 0
        for _, shape, dtype in self._buffer_specs(with_frames=with_frames):
            off = -(-off // self._ARENA_ALIGN) * self._ARENA_ALIGN + self._nbytes(shape, dtype)
        return -(-off // self._ARENA_ALIGN) * self._ARENA_ALIGN

    @staticmethod
    def _ring_piece(slot_bytes: int) -> int:
        """Piece size of a seamless ring slot (ffmp_ring.hip ring_geom; 2 MiB granularity)."""
        g = 2 << 20
        slot = -(-slot_bytes // g) * g
        return (1 << 30) if slot >= (2 << 30) else slot

    def _ring_stride(self, slot_bytes: int) -> int:
        piece = self._ring_piece(slot_bytes)
        return -(-slot_bytes // piece) * piece

    def _pick_window(self, w: Optional[int]) -> int:
        cfg, N = self.cfg, self.num_envs
        G2 = cfg.grid * cfg.grid
        plane = N * G2 * self._fes
        budget = self.hbm_budget
        if budget is not None:  # what fits: the arena (other planes, state) + W ring slots
            rest = budget - self._arena_estimate(with_frames=False)
            w_fit = rest // self._ring_stride(plane)
            if rest < 2 * plane:
                raise ValueError(f"hbm_budget {budget} B cannot hold {N} envs' planes "
                                 f"({self._arena_estimate(with_frames=False) + 2 * plane} B at W = 2)")
        if w is not None:
            if int(w) < 2:
                raise ValueError("frame_window must be >= 2")
            if budget is not None and int(w) > 2 and int(w) > w_fit:
                raise ValueError(f"frame_window={w} does not fit hbm_budget={budget} (at most {w_fit})")
            return int(w)
        if N * G2 * 12 < self.AUTOTUNE_MIN_BYTES:  # (the f32 layout's bytes: same choice for both formats)
            return 2
        other = N * G2 * ((self._pes if self.with_potential else 0) + (2 * self._pes if cfg.flow else 0) +
                          4 * self.bev_series * self._fes)
        free, _ = torch.cuda.mem_get_info(self.device)
        free += max(0, int(self.lib.ffmp_ring_pool_bytes(self.device.index)))  # parked pieces are reused
        room = self.WINDOW_HBM_FRACTION * free - other
        wmax = self.WINDOW_DEFAULT if budget is None else min(self.WINDOW_DEFAULT, w_fit)
        W = int(max(2, min(wmax, room // plane)))
        return 2 if W < 3 else W

    def _buffer_specs(self, with_frames: bool = True):
        """(name, shape, dtype) of every per-shard device buffer."""
        cfg, N = self.cfg, self.num_envs
        G, K, L = cfg.grid, cfg.n_obst, cfg.n_beams
        f32, f64, i32, b = torch.float32, torch.float64, torch.int32, torch.bool
        specs = [
            # observation planes first: the big, hot, write-streamed buffers
            ("frames", (N, 2, G, G) if getattr(self, "frame_window", 2) == 2 else (self.frame_window, N, G, G),
             self._frame_dtype),
            ("potential", (N, G, G), self._pot_dtype),
            ("flow", (N, 2, G, G), self._pot_dtype),  # float16 in the compact layout, like the potential
            # state
            ("pose", (N, 3), f64), ("goal", (N, 2), f64), ("d0", (N,), f64),
            ("obst", (N, max(K, 1), 4), f64), ("obst_r", (N, max(K, 1)), f64),
            ("t", (N,), i32), ("episode", (N,), i32), ("record", (N, cfg.record_len()), f32),
            ("err", (1,), i32),
            # small obs + outputs
            ("state_g", (N, 2), f32), ("state_v", (N, 2), f32), ("state_t", (N, 1), f32),
            ("grad", (N, 2), f32), ("lidar", (N, L), f32),
            ("reward", (N,), f32), ("done", (N,), b), ("is_goal", (N,), b), ("collision", (N,), b),
            ("truncated", (N,), b),
            # optional: post-step state before auto-reset (ffmp_state_t.term_*)
            ("term_record", (N, cfg.record_len()), f32), ("term_obs", (N, 5), f32),
            # optional: the last bev_series 4-channel BEV images of every env (ffmp_bev_image)
            ("bev", (max(getattr(self, "bev_series", 0), 1), N, 4, G, G), self._frame_dtype),
        ]
        if not self.with_potential:
            specs = [sp for sp in specs if sp[0] != "potential"]
        if not cfg.flow:
            specs = [sp for sp in specs if sp[0] != "flow"]
        if L == 0:
            specs = [sp for sp in specs if sp[0] != "lidar"]
        if not self.keep_terminal:
            specs = [sp for sp in specs if not sp[0].startswith("term_")]
        if not getattr(self, "bev_series", 0):
            specs = [sp for sp in specs if sp[0] != "bev"]
        if not with_frames:
            specs = [sp for sp in specs if sp[0] != "frames"]
        return specs

    NO_VMM = "has no virtual memory management"  # ffmp_ring_create's message (ffmp_ring.hip ring_geom)

    def _alloc_ring(self) -> bool:
        """The seamless frame ring (HIP VMM, virtual slot W aliasing slot 0), if requested and
        the device supports it; its slots are built to pair well with the potential plane the
        raster writes beside them (include/ffmp.h ffmp_ring_create)."""
        N, G = self.num_envs, self.cfg.grid
        torch.cuda.synchronize(self.device)  # the pairing probes write the potential plane on their own stream
        prev_extra = None
        try:
            partner = self.potential if self.PAIR_SLOTS else None
            if self.hbm_budget is not None:  # pairing candidates beyond need only within the budget
                slot = N * G * G * self._fes
                spare = self.hbm_budget - self._arena_used - self.frame_window * self._ring_stride(slot)
                prev_extra = _abi.set_tuning(_abi.TUNE_RING_EXTRA, 1 + max(0, spare // self._ring_piece(slot)))
            try:
                self._ring = _abi.SeamlessRing(self.device.index, (N, G, G), self.frame_window, bits=8 * self._fes,
                                               partner=partner)
            except _abi.FFMPBackendError as e:
                if self.NO_VMM in str(e):
                    raise
                # the ring's pieces come from outside torch's caching allocator: give its cached
                # blocks back to the device and try once more
                torch.cuda.empty_cache()
                self._ring = _abi.SeamlessRing(self.device.index, (N, G, G), self.frame_window, bits=8 * self._fes,
                                               partner=partner)
            self.frames = self._ring.tensor
            self.ring_meta = self._ring.info()
            if partner is not None:
                self._note_partner()
        except _abi.FFMPBackendError as e:
            # only a device without virtual memory management falls back to the wrapping ring;
            # any other failure (out of memory, a fault) is the caller's to see
            if self._seamless_req or self.NO_VMM not in str(e):
                raise
            self._seamless_req = False  # no VMM here: the wrapping ring from now on
            return False
        finally:
            if prev_extra is not None:
                _abi.set_tuning(_abi.TUNE_RING_EXTRA, prev_extra)
        self.ring = "seamless"
        self._note_hbm()
        return True

    def _note_hbm(self, extra: int = 0) -> None:
        """Track the most HBM this instance has held (hbm_peak_bytes); `extra` = bytes held beside
        the current buffers (placement tries, spacers)."""
        self.hbm_peak_bytes = max(self.hbm_peak_bytes, self.hbm_bytes() + int(extra))

    def _budget_allows(self, held_extra: int, more: int) -> bool:
        """Under hbm_budget: may the instance hold `more` bytes beside its buffers and `held_extra`?"""
        return self.hbm_budget is None or self.hbm_bytes() + held_extra + more <= self.hbm_budget

    def _alloc(self, keep_ring: bool = False):
        """All per-shard buffers, zero-initialised.  With arena=True (default) they are views
        into ONE device allocation carved at 2 MiB boundaries, planes first.  The seamless frame
        ring, when used, is its own VMM allocation, made after the arena so that its slots can
        be paired with the potential plane (keep_ring: re-allocate everything else)."""
        dev = self.device
        keep = keep_ring and self.ring == "seamless"
        want_ring = keep or self._seamless_req is not False
        if not keep:
            self.frames = None
            self._ring = None
            self.ring_meta = None
        specs = self._buffer_specs(with_frames=not want_ring)
        self.potential = None
        self.lidar = None
        self.flow = None
        self.term_record = None
        self.term_obs = None
        self.bev = None
        if self.arena:
            self._arena_offs, off = [], 0
            for _, shape, dtype in specs:
                off = -(-off // self._ARENA_ALIGN) * self._ARENA_ALIGN
                self._arena_offs.append(off)
                off += self._nbytes(shape, dtype)
            self._arena_used = -(-off // self._ARENA_ALIGN) * self._ARENA_ALIGN
            self._arena_buf = torch.zeros(max(self._arena_used, 1), dtype=torch.uint8, device=dev)
            self._carve(0, specs)
        else:
            self._arena_buf = None
            self._arena_used = 0
            for name, shape, dtype in specs:
                setattr(self, name, torch.zeros(shape, dtype=dtype, device=dev))
        if want_ring and not keep and not self._alloc_ring():
            return self._alloc()  # no VMM: the wrapping ring, frames in the arena
        if self.potential is not None:
            self.potential.zero_()  # the pairing probe wrote into it
        L = self.cfg.n_beams
        self.beam_cs = torch.as_tensor(beam_table(L), dtype=torch.float64).to(dev) if L > 0 else None
        self._note_hbm()

    @staticmethod
    def _nbytes(shape, dtype) -> int:
        n = 1
        for d in shape:
            n *= d
        return n * torch.empty((), dtype=dtype).element_size()

    def _carve(self, base: int, specs) -> None:
        """Point every buffer of `specs` into the arena, starting `base` bytes in."""
        self._arena_base = base
        for (name, shape, dtype), o in zip(specs, self._arena_offs):
            nb = self._nbytes(shape, dtype)
            setattr(self, name, self._arena_buf[base + o:base + o + nb].view(dtype).view(shape))

    # Raster launch-shape autotune (profiles/r01_placement.txt, r01_raster_tuning.txt).  The
    # raster's three concurrent 16-B store streams run anywhere from 5.7 to 7.3 TB/s depending
    # on where the planes land in HBM (fixed per allocation, identical virtual layouts) and on
    # the launch shape, and the best shape differs between allocations (e.g. 4096-cell blocks
    # 7.1-7.3 TB/s on some allocations and 5.7 on others, where 2048-cell blocks give 6.8).
    # So the shape is chosen per instance: the raster is timed on this instance's own buffers,
    # after a real reset, for each candidate, and the fastest is kept.  Results are identical
    # for every shape.
    AUTOTUNE_MIN_BYTES = 256 << 20
    # Newest-only launches (frame ring) move 2/3 of the bytes per block of a full launch, so they
    # want bigger blocks (profiles/r01_window.txt: 16384-cell blocks 7.1 TB/s vs 6.7 at 4096);
    # the two launch kinds are tuned independently from the same timed cycles.
    RASTER_SHAPES = (
        (4096, _abi.RASTER_PLAIN), (2048, _abi.RASTER_PLAIN), (2048, _abi.RASTER_PLAIN | _abi.RASTER_XCD),
        (4096, _abi.RASTER_PLAIN | _abi.RASTER_XCD), (3072, _abi.RASTER_PLAIN | _abi.RASTER_XCD),
        (2048, _abi.RASTER_NT), (4096, _abi.RASTER_NT), (2048, _abi.RASTER_NT | _abi.RASTER_XCD),
        (8192, _abi.RASTER_NT), (8192, _abi.RASTER_NT | _abi.RASTER_XCD), (16384, _abi.RASTER_NT),
        (8192, _abi.RASTER_PLAIN), (16384, _abi.RASTER_PLAIN),
        # 2-D wave tiles (compact cull box, fewer disc evaluations; identical results)
        (16384, _abi.RASTER_NT | _abi.RASTER_TILE4), (8192, _abi.RASTER_NT | _abi.RASTER_TILE4),
        (8192, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4), (16384, _abi.RASTER_NT | _abi.RASTER_TILE2),
        (16384, _abi.RASTER_NT | _abi.RASTER_TILE8), (4096, _abi.RASTER_PLAIN | _abi.RASTER_TILE4),
        # smaller tiled blocks for small planes (C2's 0.09 ms launches lose ~10 % to their last blocks)
        (4096, _abi.RASTER_NT | _abi.RASTER_TILE4), (2048, _abi.RASTER_NT | _abi.RASTER_TILE4),
        # round 3: 4,096-cell tiled blocks with the XCD remap — at C3 the fastest shape in the step loop
        # (2.265 ms against 2.345 without the remap and 2.39 for 8,192-cell blocks;
        # profiles/r03b_transient_shapes.txt, steady state)
        (4096, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4), (4096, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE2),
    )

    def _raster_gbs_steady(self, steps: int = 3) -> Dict[bool, Tuple[float, float]]:
        """Raster (GB/s, ms per launch) per launch kind (full: True, newest-only: False) in the
        real regime: whole steps (env kernel, then raster), raster launches timed with HIP
        events.  (Back-to-back rasters alone can read up to 15 % higher for some shapes than
        they sustain inside the step loop.)"""
        a = torch.full((self.num_envs,), 10, dtype=torch.int64, device=self.device)
        self.step(a)
        t = []
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(steps):
            self.step(a, timing=t)
        ev[1].record()
        torch.cuda.synchronize(self.device)
        out = {}
        for full in (True, False):
            sel = [r for r in t if r[4] == full]
            if sel:
                ms = sum(r[0].elapsed_time(r[1]) for r in sel)
                out[full] = (sum(r[3] for r in sel) / (ms * 1e-3) / 1e9, ms / len(sel))
        out["step_ms"] = ev[0].elapsed_time(ev[1]) / steps
        return out

    # Placement retries.  Two planes written in lockstep (a frame slot and the potential plane)
    # stream at ~7.1 TB/s or ~5.3-6.2 depending on where each landed in physical memory — a
    # property of the PAIR (tools/region_probe.hip, profiles/r01_ring.txt §6) — so with the
    # seamless ring one slow slot/plane pair makes one step in W ~25 % slower.  Allocating again
    # while the earlier arenas and a spacer are still held (so the allocator must return
    # different memory) often lands fast: below the threshold, up to PLACEMENT_RETRIES further
    # arenas are timed over one whole ring cycle and the fastest kept; bounded by free HBM.
    REPLACE_MIN_BYTES = 4 << 30
    PLACEMENT_FAST_GBS = 6800.0
    PLACEMENT_FAST_GBS_SEAMLESS = 7000.0  # newest-only launches only: every slot paired well
    PLACEMENT_RETRIES = 8
    PLACEMENT_SPACER = 1 << 30

    def _retry_placement(self) -> None:
        """Below the fast threshold, allocate the arena again (the seamless ring is kept: rings are
        never unmapped) while the previous ones and a growing spacer are held, time one ring
        cycle with the tuned shapes, keep the fastest; then re-tune the shapes on the winner."""
        names = [n for n, _, _ in self._buffer_specs()]  # includes "frames" (arena or ring)
        keep = [(self.placement["gbs"], self._arena_buf, {n: getattr(self, n) for n in names})]
        spacers = []
        tries = [round(self.placement["gbs"], 1)]
        fast = self.PLACEMENT_FAST_GBS_SEAMLESS if self.ring == "seamless" else self.PLACEMENT_FAST_GBS
        for k in range(self.PLACEMENT_RETRIES):
            if max(c[0] for c in keep) >= fast:
                break
            free, _ = torch.cuda.mem_get_info(self.device)
            if free < 1.2 * self._arena_buf.numel() + (k + 1) * self.PLACEMENT_SPACER + (1 << 30):
                break
            held = sum(c[1].numel() for c in keep[1:]) + sum(t.numel() for t in spacers)
            if not self._budget_allows(held, self._arena_buf.numel() + (k + 1) * self.PLACEMENT_SPACER):
                break
            spacers.append(torch.empty((k + 1) * self.PLACEMENT_SPACER, dtype=torch.uint8, device=self.device))
            self._alloc(keep_ring=True)
            self._note_hbm(held + spacers[-1].numel())
            self._build_structs()
            gbs = self._placement_gbs()
            tries.append(round(gbs, 1))
            keep.append((gbs, self._arena_buf, {n: getattr(self, n) for n in names}))
        best = max(range(len(keep)), key=lambda i: keep[i][0])
        _, buf, views = keep[best]
        self._arena_buf = buf
        for n, v in views.items():
            setattr(self, n, v)
        self._build_structs()
        del keep, spacers, views, buf
        torch.cuda.empty_cache()
        if best > 0:
            self._autotune_raster()
        self.placement = dict(self.placement, placement_tries=tries, placement_kept=best)

    # Slot repair (seamless ring).  The pairing probe at ring creation predicts most, not all,
    # slow slot/potential pairings; the step loop itself is the judge: time every slot's
    # newest-only raster over two ring cycles (after SLOT_WARMUP_CYCLES untimed ones) and rebuild
    # the ring with new pieces for slots more than SLOW_SLOT above the fastest (ffmp_ring_rebuild),
    # up to REPAIR_ROUNDS times, keeping the rebuilt ring only if its cycle is faster; a reverted
    # rebuild does not end the repair — the next round draws other pieces (round 6: one C3 box kept a
    # slot 15 % slow after its single rebuild came out worse, 13.41 vs 13.71 M on the same box,
    # profiles/r06g_bench_default_*.json).  (The 12 % threshold of rounds 1-3 guarded against rebuilds
    # judged on post-idle timings; with the warm-up, 6 %: profiles/r04h_slot_repair.txt.)
    SLOW_SLOT = 1.06
    REPAIR_ROUNDS = 3
    PAIR_SLOTS = True  # build the ring's slots from pieces probed against the potential plane

    # untimed ring cycles before the slot timing: the timing follows host work (construction, a
    # rebuild's pairing probes) that left the GPU idle, and after such a gap the raster runs slow
    # for about one ring cycle while the GPU warms up again (profiles/r03b_transient_*.txt); timed
    # straight after a rebuild, kept slots read 4-7 % slow and good rebuilds were reverted
    # (profiles/r04h_slot_repair.txt)
    SLOT_WARMUP_CYCLES = 2

    def _slot_ms(self) -> Dict[int, float]:
        """Median newest-only raster ms per physical slot written, over two ring cycles."""
        W = self.frame_window
        self.reset()
        a = torch.full((self.num_envs,), 10, dtype=torch.int64, device=self.device)
        for _ in range(self.SLOT_WARMUP_CYCLES * W):
            self.step(a)
        t = []
        for _ in range(2 * W):
            self.step(a, timing=t)
        torch.cuda.synchronize(self.device)
        per: Dict[int, list] = {}
        S = self.pipeline_slices  # timing entries per step (one raster launch per env slice)
        for k in range(len(t) // S):
            per.setdefault(self._slot_written(k), []).append(sum(r[0].elapsed_time(r[1]) for r in t[k * S:(k + 1) * S]))
        self._clear_after_tuning()
        return {i: float(np.median(v)) for i, v in per.items()}

    def _slot_written(self, k: int) -> int:
        """Physical ring slot whose newest frame step k (0-based) after a full reset writes: the
        reset leaves the window at [0, 1], step k slides it to [k+1, k+2] and writes the newest
        frame, virtual slot k+2 -> physical (k+2) % W (virtual slot W is slot 0)."""
        return (k + 2) % self.frame_window

    # Partner relocation (seamless ring).  The ring's pieces are probed against the potential
    # plane; when no probe reaches PAIR_FAST_GBS the plane itself sits where nothing pairs well
    # (round-1 C5 and some C3 boxes: every probe 4.9-5.5 TB/s).  Then the arena (with the potential
    # plane) is allocated again elsewhere — the earlier arenas and a growing spacer stay held so
    # the allocator must return different memory — and a ring is paired against the new plane
    # (the losing rings' pieces return to the pool and are probed again first); the pair with the
    # fastest probe is kept.
    # Small planes too (round 2, profiles/r02_env_chain.txt): at C2 (0.5 GB of planes, 256-MiB
    # ring pieces) every first probe paired at 5.3-5.6 TB/s and the raster ran 0.106 ms; the third
    # relocation found a 6.8 TB/s pair on each of three fresh runs, raster 0.089 ms (+16 % env-steps/s).
    # Below REPLACE_MIN_BYTES a try is cheap (a < 4 GiB arena, a few 256-MiB probes), so more are allowed.
    PAIR_FAST_GBS = 6200.0  # ffmp_ring.hip kPairFastGBs
    PARTNER_TRIES = 3
    PARTNER_TRIES_SMALL = 6
    RELOCATE_MIN_BYTES = 512 << 20  # planes of C2 size up (the ring pairs pieces of >= 256 MiB)

    def _relocate_partner(self, max_tries: int) -> None:
        meta = self.ring_meta or {}
        if not meta.get("pair_probes") or meta.get("pair_gbs_max", 0.0) >= self.PAIR_FAST_GBS:
            return
        names = [n for n, _, _ in self._buffer_specs(with_frames=False)]

        def snap():
            return {"gbs": self.ring_meta["pair_gbs_max"], "arena": self._arena_buf, "ring": self._ring,
                    "meta": self.ring_meta, "views": {n: getattr(self, n) for n in names}}

        best = snap()
        tries, held = [best["gbs"]], []
        ring_bytes = self.frame_window * self._ring.slot_stride
        for k in range(max_tries):
            free, _ = torch.cuda.mem_get_info(self.device)
            if free < self._arena_used + (k + 1) * self.PLACEMENT_SPACER + ring_bytes + (16 << 30):
                break
            # under hbm_budget: the arenas held so far (the best's among them) + this try's spacer,
            # arena and ring beside the best ring
            held_b = sum(t.numel() for t in held)
            if self.hbm_budget is not None and ring_bytes + max(held_b, self._arena_used) + self._arena_used + \
                    (k + 1) * self.PLACEMENT_SPACER + ring_bytes > self.hbm_budget:
                break
            held.append(self._arena_buf)
            held.append(torch.empty((k + 1) * self.PLACEMENT_SPACER, dtype=torch.uint8, device=self.device))
            self._ring = self.frames = None  # the best ring stays referenced by `best`
            try:
                self._alloc()
            except _abi.FFMPBackendError:
                break
            if self.ring != "seamless" or self._ring is None:
                break
            self.hbm_peak_bytes = max(self.hbm_peak_bytes, ring_bytes + sum(t.numel() for t in held) +
                                      self._arena_used + self.frame_window * self._ring.slot_stride)
            cur = snap()
            tries.append(cur["gbs"])
            if cur["gbs"] > best["gbs"]:
                best = cur
            cur = None
            if best["gbs"] >= self.PAIR_FAST_GBS:
                break
        self._arena_buf, self._ring, self.ring = best["arena"], best["ring"], "seamless"
        for n, v in best["views"].items():
            setattr(self, n, v)
        self.frames = self._ring.tensor
        self._arena_used = self._arena_buf.numel()
        torch.cuda.synchronize(self.device)
        del held
        self.potential.zero_()
        self.frames[:self.frame_window].zero_()
        self.ring_meta = dict(best["meta"], partner_tries=[round(g, 1) for g in tries])
        best = None
        torch.cuda.empty_cache()

    def _adopt_ring_tensor(self) -> None:
        self.frames = self._ring.tensor
        self.potential.zero_()
        self._build_structs()

    def _repair_slots(self) -> None:
        """Rebuild slow slots and keep whichever ring cycles faster: a rebuild maps every slot at
        new addresses and has left kept slots slower than before (round-1 repair logs), so the
        old ring stays alive until the new one has been timed (SeamlessRing.rebuild keep_old)."""
        history = []
        ms = self._slot_ms()
        for _ in range(self.REPAIR_ROUNDS):
            fast = min(ms.values())
            slow = [i for i, v in ms.items() if v > self.SLOW_SLOT * fast]
            history.append({"slot_ms": [round(ms[i], 3) for i in sorted(ms)], "slow": slow})
            if not slow:
                break
            # the tuning launches (and _clear_after_tuning's memsets) must be done before the
            # rebuild's pairing probes write the potential plane on their own stream
            torch.cuda.synchronize(self.device)
            try:
                self._ring.rebuild(sum(1 << i for i in slow), partner=self.potential, keep_old=True)
            except _abi.FFMPBackendError as err:
                # the rebuild maps the new pieces beside the old ring: with the HBM shared (several
                # ranks on one device) it can run out; the current ring is whole and stays, and the
                # pieces the rebuild took went back to the pool (trimmed below / in __init__)
                history.append({"skipped": str(err)[:200]})
                break
            self._adopt_ring_tensor()
            new = self._slot_ms()
            if sum(new.values()) < sum(ms.values()):
                torch.cuda.synchronize(self.device)
                self._ring.drop_previous()
                ms = new
            else:  # the rebuilt ring cycles slower: back to the previous one, then another round
                history.append({"slot_ms": [round(new[i], 3) for i in sorted(new)], "reverted": True})
                torch.cuda.synchronize(self.device)
                self._ring.revert()
                self._adopt_ring_tensor()
                self._clear_after_tuning()
        else:  # every round rebuilt: the kept ring's timing (slots still slow if the last rebuilds lost)
            fast = min(ms.values())
            history.append({"slot_ms": [round(ms[i], 3) for i in sorted(ms)],
                            "slow": [i for i, v in ms.items() if v > self.SLOW_SLOT * fast]})
        self.ring_meta = dict(self.ring_meta or {}, **self._ring.info(), repair=history)

    def tuning(self) -> dict:
        """The launch choices of this instance (pass as FFMPVec(tuning=...) to skip the autotune)."""
        return {"shape": list(self.raster_shape), "shape_newest": list(self.raster_shape_newest),
                "fused": bool(self.fused), "fused_flags": int(self.fused_flags)}

    def _apply_tuning(self, t: dict) -> None:
        self.raster_shape = tuple(t["shape"])
        self.raster_shape_newest = tuple(t.get("shape_newest", t["shape"]))
        self.fused = bool(t.get("fused", False)) and self.pipeline_slices == 1 and self._fused_req is not False
        self.fused_flags = int(t.get("fused_flags", _abi.RASTER_NT))
        self.placement = {"shape": {"cells_per_block": self.raster_shape[0], "flags": self.raster_shape[1]},
                          "shape_newest": {"cells_per_block": self.raster_shape_newest[0],
                                           "flags": self.raster_shape_newest[1]},
                          "from": "tuning", "fused": {"chosen": self.fused, "flags": self.fused_flags}}

    def _tune_steps(self) -> int:
        """Timed steps per measurement: >= ~10 ms of raster, in whole ring cycles — the wrapping
        ring's W-1 steps (one full raster), or the seamless ring's W steps: every slot is written
        once, and the potential plane streams beside each slot at its own rate (one slow
        slot/plane pairing makes one step in W ~25 % slower, profiles/r01_ring.txt §6), so a
        placement check must see all of them."""
        plane_bytes = self.state_m.numel() * (self._fes + (self._pes / 2 if self.with_potential else 0.0) +
                                              (float(self._pes) if self.flow is not None else 0.0))
        steps = 3 if plane_bytes >= (8 << 30) else 12
        cyc = {"wrap": self.frame_window - 1, "seamless": self.frame_window}.get(self.ring, 1)
        return -(-steps // cyc) * cyc

    def _cycle_gbs(self, ms_full: Optional[float], ms_newest: Optional[float]) -> float:
        """Raster bandwidth of one ring cycle from per-launch times of the two kinds: one full
        launch + W-2 newest-only ones (wrapping ring), full launches only (W = 2) or newest-only
        ones only (seamless ring)."""
        n_new, n_full = self.frame_window - 2, 1
        if self.ring == "seamless":
            n_new, n_full = 1, 0
        b = n_full * self._raster_bytes(self.num_envs, True) + n_new * self._raster_bytes(self.num_envs, False)
        ms = (ms_full if n_full else 0.0) + (n_new * ms_newest if n_new else 0.0)
        return b / (ms * 1e-3) / 1e9

    def _clear_after_tuning(self) -> None:
        if self._arena_buf is not None:
            self._arena_buf.zero_()
        if self.ring == "seamless":
            self.frames[:self.frame_window].zero_()
        self._needs_reset = True

    def _autotune_raster(self) -> None:
        self.reset()  # a real state (a zeroed record would stack every disc on the robot cell)
        results = []
        steps = self._tune_steps()
        for shape in self._shape_candidates():
            self.raster_shape = self.raster_shape_newest = shape
            results.append((self._raster_gbs_steady(steps), shape))
        best = {}
        for kind in (True, False):
            got = [(r[kind][0], r[kind][1], shape) for r, shape in results if kind in r]
            if got:
                best[kind] = max(got)
        if True in best:
            self.raster_shape = best[True][2]
        else:  # seamless ring: steps never write both frames; resets use the newest-only winner
            self.raster_shape = best[False][2]
        self.raster_shape_newest = best[False][2] if False in best else self.raster_shape
        gbs = self._cycle_gbs(best[True][1] if True in best else None, best[False][1] if False in best else None)
        fused = self._tune_fused(steps)
        self.placement = {"shape": {"cells_per_block": self.raster_shape[0], "flags": self.raster_shape[1]},
                          "shape_newest": ({"cells_per_block": self.raster_shape_newest[0],
                                            "flags": self.raster_shape_newest[1]} if False in best else None),
                          "gbs": round(gbs, 1),
                          "candidates": [[c, f] + [round(r[k][0], 1) for k in (True, False) if k in r]
                                         for r, (c, f) in results],
                          "fused": fused}
        self._clear_after_tuning()

    # Fused-step candidates (ffmp_step_fused flags; a block is a whole plane, so no cells/block)
    FUSED_FLAGS = (
        _abi.RASTER_NT, _abi.RASTER_PLAIN, _abi.RASTER_NT | _abi.RASTER_XCD, _abi.RASTER_PLAIN | _abi.RASTER_XCD,
        _abi.RASTER_NT | _abi.RASTER_TILE4, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4,
        _abi.RASTER_PLAIN | _abi.RASTER_TILE4, _abi.RASTER_NT | _abi.RASTER_TILE2,
        _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE2, _abi.RASTER_NT | _abi.RASTER_TILE8,
    )

    # The compact format (obs_format="u8f16") writes 3 bytes per cell and is bound by the per-task
    # cull / wall / index work rather than by HBM (tools/compact_probe.py): 16 cells per lane
    # (1024-cell wave tasks) by default, tiles R x 1024/R; NARROW = the 4-cells-per-lane kernel.
    # (round 2: the 16-cells-per-lane tiles hoist their columns' work out of the tile loop;
    # tools/compact_shapes.py: whole-plane blocks, 4- or 16-cell lanes, 1.46-1.55 ms at C3)
    COMPACT_SHAPES = (
        (65536, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_NARROW),
        (32768, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_NARROW),
        (16384, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_NARROW),
        (65536, _abi.RASTER_PLAIN | _abi.RASTER_TILE16), (32768, _abi.RASTER_NT | _abi.RASTER_TILE16),
        (16384, _abi.RASTER_NT | _abi.RASTER_TILE16), (65536, _abi.RASTER_NT | _abi.RASTER_TILE4),
        (16384, _abi.RASTER_NT | _abi.RASTER_TILE8), (16384, _abi.RASTER_PLAIN | _abi.RASTER_TILE16),
        (32768, _abi.RASTER_PLAIN | _abi.RASTER_TILE4 | _abi.RASTER_NARROW),
        # round 3: 4-cell lanes in 2 x 128-cell tiles or 256-cell rows, so that a wave's uint8 frame
        # stores cover whole 128-byte lines (TILE4's 64-cell rows write half lines: PMC 1.02x)
        (32768, _abi.RASTER_NT | _abi.RASTER_TILE2 | _abi.RASTER_NARROW),
        (65536, _abi.RASTER_NT | _abi.RASTER_TILE2 | _abi.RASTER_NARROW),
        (32768, _abi.RASTER_NT | _abi.RASTER_NARROW),
        # round 3: 8 cells per lane (an 8-B frame and a 16-B potential store per lane), 4 x 128-cell
        # tiles, 6 waves per SIMD: 0.954-0.985 ms against the 4-cell tiles' 1.00-1.03 at C3
        # (profiles/r03b_ct8_shapes.txt)
        (65536, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_MID8),
        (32768, _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_MID8),
        (65536, _abi.RASTER_NT | _abi.RASTER_TILE8 | _abi.RASTER_MID8),
        (65536, _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE4 | _abi.RASTER_MID8),
    )
    COMPACT_FUSED_FLAGS = (
        _abi.RASTER_NT | _abi.RASTER_TILE16, _abi.RASTER_NT | _abi.RASTER_TILE8, _abi.RASTER_NT | _abi.RASTER_TILE4,
        _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_NARROW, _abi.RASTER_PLAIN | _abi.RASTER_TILE16,
        _abi.RASTER_NT | _abi.RASTER_XCD | _abi.RASTER_TILE16, _abi.RASTER_NT,
        _abi.RASTER_NT | _abi.RASTER_TILE2 | _abi.RASTER_NARROW,
        _abi.RASTER_NT | _abi.RASTER_TILE4 | _abi.RASTER_MID8,
    )

    XCD_SHAPES = True  # autotune candidates include the XCD-aware block remap

    def _shape_candidates(self):
        shapes = self.COMPACT_SHAPES if self.obs_format == "u8f16" else self.RASTER_SHAPES
        return [sh for sh in shapes if self.XCD_SHAPES or not sh[1] & _abi.RASTER_XCD]

    def _fused_candidates(self):
        flags = self.COMPACT_FUSED_FLAGS if self.obs_format == "u8f16" else self.FUSED_FLAGS
        return [f for f in flags if self.XCD_SHAPES or not f & _abi.RASTER_XCD]

    def _tune_fused(self, steps: int) -> Optional[dict]:
        """Time whole steps of the two-launch path (the tuned raster shapes) against the fused
        step for each FUSED_FLAGS candidate; keep the faster (fused=None), or the best fused flags
        (fused=True)."""
        if self._fused_req is False or self.pipeline_slices > 1:
            self.fused = False
            return None
        self.fused = False
        sep = self._raster_gbs_steady(steps)["step_ms"]
        self.fused = True
        res = []
        for f in self._fused_candidates():
            self.fused_flags = f
            res.append((self._raster_gbs_steady(steps)["step_ms"], f))
        best_ms, best_f = min(res)
        self.fused_flags = best_f
        self.fused = bool(self._fused_req) or best_ms < 0.995 * sep
        return {"chosen": self.fused, "two_launch_step_ms": round(sep, 4), "fused_step_ms": round(best_ms, 4),
                "flags": best_f, "candidates": [[f, round(m, 4)] for m, f in res]}

    def _recheck_fused(self) -> None:
        """The one- or two-launch decision again, on the repaired ring.  _autotune_raster makes it
        before the slot repair, whose rebuilt slots change the step time by 5-10 %, and the two
        kinds are within ~2 % of each other at C3: on three fresh runs of one box the pre-repair
        choice kept the two-launch step at 2.48-2.50 ms where the one-launch step ran 2.44 ms
        (profiles/r02_fused_recheck.txt).  Two alternating rounds of two ring cycles each, the
        better of each kind; the autotune's best fused flags; the two-launch step only if it is
        0.5 % faster."""
        tf = (self.placement or {}).get("fused")
        if self._fused_req is not None or self.pipeline_slices > 1 or not tf:
            return
        self.reset()
        steps = 2 * self._tune_steps()
        rounds = 2
        if max(tf.get("two_launch_step_ms", 1.0), tf.get("fused_step_ms", 1.0)) < self.SHORT_STEP_MS:
            # short steps (C2: ~0.1 ms) vary by several % between rounds of a few steps, and the
            # one- and two-launch steps are within that of each other (a 2-round pick
            # kept a path 3 % slower): more and longer alternating rounds, compared by their medians
            rounds = self.SHORT_STEP_ROUNDS
            cyc = max(1, self.graph_period())
            steps = max(steps, -(-self.SHORT_STEP_MIN_STEPS // cyc) * cyc)
        ms = {False: [], True: []}
        for _ in range(rounds):
            for kind in (False, True):
                self.fused = kind
                self.fused_flags = tf["flags"]
                ms[kind].append(self._raster_gbs_steady(steps)["step_ms"])
        pick = min if rounds <= 2 else (lambda v: float(np.median(v)))
        sep, fus = pick(ms[False]), pick(ms[True])
        # ties go to the one-launch step: on the repaired ring it was the faster one on every box
        # measured (0.3-1.4 %), the two-launch step only ahead on poorly paired rings
        self.fused = not (sep < 0.995 * fus)
        self._clear_after_tuning()
        self.placement = dict(self.placement, fused=dict(tf, chosen=self.fused, recheck={
            "two_launch_step_ms": round(sep, 4), "fused_step_ms": round(fus, 4), "rounds": rounds,
            "steps_per_round": steps, "statistic": "min" if rounds <= 2 else "median",
            "two_launch_rounds_ms": [round(v, 4) for v in ms[False]],
            "fused_rounds_ms": [round(v, 4) for v in ms[True]]}))

    SHORT_STEP_MS = 0.5        # below this, the one- / two-launch recheck takes SHORT_STEP_ROUNDS rounds ...
    SHORT_STEP_ROUNDS = 8      # ... alternating, of >= SHORT_STEP_MIN_STEPS steps each (whole ring cycles)
    SHORT_STEP_MIN_STEPS = 50

    def _placement_gbs(self) -> float:
        """Cycle bandwidth of the current buffers with the current launch shapes."""
        self.reset()
        r = self._raster_gbs_steady(self._tune_steps())
        gbs = self._cycle_gbs(r[True][1] if True in r else None, r[False][1] if False in r else None)
        self._clear_after_tuning()
        return gbs

    def _build_structs(self):
        self._cfg_c = _abi.make_cfg(self.cfg, _ptr(self.beam_cs) or 0)
        self._state_c = _abi.StateT(self.pose.data_ptr(), self.goal.data_ptr(), self.d0.data_ptr(),
                                    self.obst.data_ptr(), self.obst_r.data_ptr(), self.t.data_ptr(),
                                    self.episode.data_ptr(), self.record.data_ptr(), self.err.data_ptr(),
                                    _ptr(self.term_record), _ptr(self.term_obs))
        G2 = self.cfg.grid * self.cfg.grid
        self._obs_c = _abi.ObsT(self.state_m.data_ptr(), self.state_g.data_ptr(), self.state_v.data_ptr(),
                                self.state_t.data_ptr(), _ptr(self.potential), self.grad.data_ptr(),
                                _ptr(self.lidar), _ptr(self.flow), *self._sm_strides(), self._fmt)
        self._out_c = _abi.OutT(self.reward.data_ptr(), self.done.data_ptr(), self.is_goal.data_ptr(),
                                self.collision.data_ptr(), self.truncated.data_ptr())
        self._build_slices()

    # Optional pipelined step (pipeline=S > 1): the env kernel of slice s+1 runs on a
    # high-priority side stream while the raster of slice s runs on the caller's stream.
    # Results are identical; on MI355X it did not pay (the raster fills every CU, the slices
    # add kernel tails), so the default is the serial step.

    def _build_slices(self):
        N, S = self.num_envs, self.pipeline_slices
        bounds = [N * k // S for k in range(S + 1)]

        def off(t, e0):
            return None if t is None else t.data_ptr() + e0 * t.stride(0) * t.element_size()

        self._slices = []
        for k in range(S):
            a, n = bounds[k], bounds[k + 1] - bounds[k]
            st = _abi.StateT(off(self.pose, a), off(self.goal, a), off(self.d0, a), off(self.obst, a),
                             off(self.obst_r, a), off(self.t, a), off(self.episode, a), off(self.record, a),
                             self.err.data_ptr(), off(self.term_record, a), off(self.term_obs, a))
            ob = _abi.ObsT(off(self.state_m, a), off(self.state_g, a), off(self.state_v, a), off(self.state_t, a),
                           off(self.potential, a), off(self.grad, a), off(self.lidar, a), off(self.flow, a), 0, 0,
                           self._fmt)
            out = _abi.OutT(off(self.reward, a), off(self.done, a), off(self.is_goal, a), off(self.collision, a),
                            off(self.truncated, a))
            self._slices.append((a, n, st, ob, out, off(self.record, a)))
        if S > 1 and getattr(self, "_side", None) is None:
            lo, hi = torch.cuda.Stream.priority_range()
            self._side = torch.cuda.Stream(self.device, priority=hi)  # env kernels first
            self._ev_go = torch.cuda.Event()
        if S > 1 and len(getattr(self, "_ev_slice", ())) != S:
            self._ev_slice = [torch.cuda.Event() for _ in range(S)]

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # ------------------------------------------------------------ frame window
    @property
    def state_m(self) -> torch.Tensor:
        """(N, 2, G, G) [older, newest] view of the frame window (contiguous iff W == 2)."""
        if self.frame_window == 2:
            return self.frames
        return self.frames[self._wpos:self._wpos + 2].transpose(0, 1)

    def _sm_strides(self):
        """(env stride, frame stride) of state_m in elements, for ffmp_obs_t."""
        G2 = self.cfg.grid * self.cfg.grid
        if self.frame_window == 2:
            return (2 * G2, G2)
        return (G2, self.frames.stride(0))

    # Seamless ring, wrap step (pair [W-1, W]): the newest frame goes to physical slot 0, which
    # virtual slots 0 and W both map.  WRAP_VIA_ALIAS False: the raster writes it through slot
    # 0's own addresses (negative frame stride from slot W-1); the state_m view still reads it
    # through slot W.  Same bytes either way.
    WRAP_VIA_ALIAS = True

    def _set_window(self, p: int) -> None:
        self._wpos = p
        self._obs_c.state_m = self.frames.data_ptr() + p * self.frames.stride(0) * self._fes
        if self.ring == "seamless":
            W, fs = self.frame_window, self.frames.stride(0)
            wrap = p == W - 1 and not self.WRAP_VIA_ALIAS
            self._obs_c.state_m_frame_stride = -(W - 1) * fs if wrap else fs

    def _note_window(self, full: bool) -> None:
        """Frame history after a raster at the current window: the newest frame's slot first;
        a full raster also rewrote the older slot (with the previous newest frame)."""
        if self.frame_window == 2:
            return
        W = self.frame_window
        new, old = (self._wpos + 1) % W, self._wpos % W
        prev = self._hist
        if full:
            self._hist = [new, old] + [s for s in prev[1:] if s not in (new, old)]
        else:
            self._hist = [new] + [s for s in prev if s != new]
        del self._hist[W:]
        if len(self._hist) < len(prev) + 1:
            # a frame of the history was overwritten: lags beyond the list are no longer
            # guaranteed to be clamped away
            self._hist_from_reset = False

    @property
    def max_temporal_frames(self) -> int:
        """The largest k temporal_maps(k) can serve at every step: W for the seamless ring and the
        contiguous pair, W - 1 for the wrapping ring (its wrap re-rasters the newest frame into slot 0,
        so after the first wrap it holds W - 1 distinct frames)."""
        return self.frame_window - 1 if self.ring == "wrap" else self.frame_window

    def _bev_push(self, advance: bool, restart: bool = False) -> None:
        """Write the current BEV image of every env into the ring (bev_series): a new slot after a
        step (advance), the current one again after a re-raster or masked reset, slot 0 after a full
        reset (restart: every env's older lags are clamped away)."""
        if self.bev is None:
            return
        S = self.bev.shape[0]
        if restart:
            self._bev_pos, self._bev_hist, self._bev_from_reset = 0, [0], True
        elif advance:
            self._bev_pos = (self._bev_pos + 1) % S
            self._bev_hist = ([self._bev_pos] + self._bev_hist)[:S]
        elif not self._bev_hist:
            self._bev_hist = [self._bev_pos]
        G2 = self.cfg.grid * self.cfg.grid
        sm = self.state_m
        with torch.cuda.device(self.device):
            self._bev_launch(sm, G2)

    def _bev_launch(self, sm: torch.Tensor, G2: int) -> None:
        _abi.check(self.lib.ffmp_bev_image(self.num_envs, 1 if self.obs_format == "u8f16" else 0,
                                           sm[:, 1].data_ptr(), sm.stride(0), self.flow.data_ptr(), G2,
                                           float(np.float32(self.cfg.obst_vmax)), self.bev[self._bev_pos].data_ptr(),
                                           4 * G2, self._stream()), "ffmp_bev_image")

    def bev_maps(self, k: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """make_temporal_maps over the last k 4-channel BEV images (bev_series): (N, 4k, G, G),
        oldest image first, each [occupancy, R, G, B] (include/ffmp.h ffmp_bev_image), every env's
        lags clamped to its episode start as in temporal_maps (is_first refills map_memory) — the
        reference's INPUT_CHANNELS = 12 option at k = 3 (train.py:66, ffmp.py:16).  Gathered by
        ffmp_temporal_maps from the ring into `out` (or a new tensor; frames' dtype)."""
        self._check_open()
        if self.bev is None:
            raise RuntimeError("bev_maps() needs FFMPVec(..., bev_series=k)")
        S = self.bev.shape[0]
        k = S if k is None else int(k)
        if not 1 <= k <= S:
            raise ValueError(f"k must be in [1, {S}] (bev_series={S})")
        if self._needs_reset:
            raise RuntimeError("call reset() before bev_maps()")
        if len(self._bev_hist) < k and not self._bev_from_reset:
            raise RuntimeError(f"the BEV ring holds {len(self._bev_hist)} known images since the last reload; "
                               f"bev_maps({k}) needs {k} (step {k - len(self._bev_hist)} more times, or reset())")
        N, G = self.num_envs, self.cfg.grid
        plane = 4 * G * G
        hist = self._bev_hist
        offs = [hist[min(d, len(hist) - 1)] * N * plane for d in range(k)]
        if out is None:
            out = torch.empty(N, 4 * k, G, G, dtype=self.bev.dtype, device=self.device)
        elif out.shape != (N, 4 * k, G, G) or out.dtype != self.bev.dtype or not out.is_contiguous() \
                or out.device != self.device:
            raise ValueError(f"out must be a contiguous {self.bev.dtype} tensor of shape {(N, 4 * k, G, G)} on {self.device}")
        lag = (C.c_int64 * k)(*offs)
        _abi.check(self.lib.ffmp_temporal_maps(N, self.bev.data_ptr(), lag, k, plane, plane, self._fes,
                                               self.t.data_ptr(), out.data_ptr(), self._stream()), "ffmp_temporal_maps")
        return out

    def temporal_maps(self, k: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """make_temporal_maps (src/train.py:474-486) over the last k frames: (N, k, G, G), oldest
        first, each env's lags clamped to its episode start (is_first refills the reference's
        map_memory with the first frame) — the reference's INPUT_CHANNELS = k with a mono BEV
        image (train.py:66-69).  k <= 2: a view of state_m.  k > 2: gathered from the frame ring
        (k <= frame_window) by ffmp_temporal_maps into `out` (or a new tensor)."""
        self._check_open()
        k = int(k)
        if k < 1:
            raise ValueError("k must be >= 1")
        if k <= 2 and out is None:
            return self.state_m[:, 2 - k:]
        if k > self.max_temporal_frames or k > _abi.MAX_SERIES:
            raise ValueError(f"temporal_maps({k}) needs at most {self.max_temporal_frames} frames here "
                             f"(frame_window={self.frame_window}, ring={self.ring}: a wrapping ring re-rasters "
                             f"its newest frame into slot 0 and keeps W - 1 distinct frames; at most "
                             f"{_abi.MAX_SERIES})")
        if self._needs_reset:
            raise RuntimeError("call reset() before temporal_maps()")
        N, G = self.num_envs, self.cfg.grid
        if self.frame_window == 2:
            offs = [G * G, 0]  # contiguous (N, 2, G, G): newest, older
            env_stride = 2 * G * G
        else:
            if len(self._hist) < k and not self._hist_from_reset:
                raise RuntimeError(f"the frame ring holds {len(self._hist)} known frames since the last reload; "
                                   f"temporal_maps({k}) needs {k} (step {k - len(self._hist)} more times, or reset())")
            # lags the ring has not seen since a full reset are never read (every env's lag is
            # clamped to its steps since that reset): any valid slot stands in
            offs = [self._hist[min(d, len(self._hist) - 1)] * self.frames.stride(0) for d in range(k)]
            env_stride = G * G
        offs = (offs + [offs[-1]] * k)[:k]
        if out is None:
            out = torch.empty(N, k, G, G, dtype=self.frames.dtype, device=self.device)
        elif out.shape != (N, k, G, G) or out.dtype != self.frames.dtype or not out.is_contiguous() \
                or out.device != self.device:
            raise ValueError(f"out must be a contiguous {self.frames.dtype} tensor of shape {(N, k, G, G)} on {self.device}")
        lag = (C.c_int64 * k)(*offs)
        _abi.check(self.lib.ffmp_temporal_maps(N, self.frames.data_ptr(), lag, k, env_stride, G * G, self._fes,
                                               self.t.data_ptr(), out.data_ptr(), self._stream()), "ffmp_temporal_maps")
        return out

    def _raster_bytes(self, n: int, full: bool) -> int:
        """Algorithmic bytes of one raster launch over n envs (excluding the older frames of envs
        reset during a newest-only launch: one frame each, added by bench.py from the episode counts)."""
        G2 = self.cfg.grid * self.cfg.grid
        per = (2 if full else 1) * self._fes * G2 + (self._pes * G2 if self.potential is not None else 0) + \
            (2 * self._pes * G2 if self.flow is not None else 0) + 4 * self.cfg.record_len()
        return n * per

    def _raster_launch(self, full: bool, mask=None, timing: Optional[list] = None) -> None:
        self._check_open()
        cpb, flags = self.raster_shape if full else self.raster_shape_newest
        flags |= 0 if full else _abi.RASTER_NEWEST
        if timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _abi.check(self.lib.ffmp_raster_ex(C.byref(self._cfg_c), self.num_envs, self.record.data_ptr(), _ptr(mask),
                                           C.byref(self._obs_c), cpb, flags, self._stream()), "ffmp_raster")
        if timing is not None:
            e1.record()
            timing.append((e0, e1, self.num_envs, self._raster_bytes(self.num_envs, full), full))

    # --------------------------------------------------------------- gym API
    @property
    def obs(self) -> Dict[str, torch.Tensor]:
        d = {"state_m": self.state_m, "state_g": self.state_g, "state_v": self.state_v, "state_t": self.state_t,
             "grad": self.grad}
        if self.potential is not None:
            d["potential"] = self.potential
        if self.lidar is not None:
            d["lidar"] = self.lidar
        if self.flow is not None:
            d["flow"] = self.flow
        return d

    def _obs_out(self, copy: bool):
        o = self.obs
        return {k: v.clone() for k, v in o.items()} if copy else o

    def reset(self, seed: Optional[int] = None, mask: Optional[torch.Tensor] = None, copy: bool = False):
        """Reset all envs (mask None: new episodes 0 from `seed`) or only masked ones."""
        self._check_open()
        with torch.cuda.device(self.device):
            if seed is not None:
                self._set_cfg(self.cfg.replace(seed=int(seed)))
            m = None
            if mask is not None:
                m = mask.to(device=self.device, dtype=torch.bool).contiguous().view(torch.uint8)
                if m.numel() != self.num_envs:
                    raise ValueError("mask must have num_envs elements")
            initial = 1 if (mask is None) else 0
            s = self._stream()
            if mask is None:
                self._set_window(0)
                self._hist, self._hist_from_reset = [], True
                self._note_window(True)
            _abi.check(self.lib.ffmp_reset(C.byref(self._cfg_c), self.num_envs, self.env_offset, _ptr(m), initial,
                                           C.byref(self._state_c), C.byref(self._obs_c), s), "ffmp_reset")
            self._raster_launch(True, m)
            self._mask_keepalive = m
            self._bev_push(advance=False, restart=mask is None)
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
        self._check_open()
        a = self._actions(actions)
        self._act_keepalive = a
        _abi.check(self.lib.ffmp_step_state(C.byref(self._cfg_c), self.num_envs, self.env_offset, a.data_ptr(),
                                            C.byref(self._state_c), C.byref(self._obs_c), C.byref(self._out_c),
                                            self._stream()), "ffmp_step_state")

    def raster(self, mask: Optional[torch.Tensor] = None) -> None:
        """Re-raster the current observation (both frames, potential, flow) from the record."""
        self._check_open()
        m = None if mask is None else mask.to(device=self.device, dtype=torch.bool).contiguous().view(torch.uint8)
        self._raster_launch(True, m)
        self._bev_push(advance=False)

    def _next_window(self) -> bool:
        """Slide the [older, newest] pair by one slot for the next raster; True if that raster
        must write both frames (the wrapping ring's wrap, or W = 2)."""
        p = self._wpos + 1
        if self.ring == "seamless":  # virtual slot W is slot 0: the pair slides forever
            full = False
            p %= self.frame_window
        else:
            full = p > self.frame_window - 2
        self._set_window(0 if full else p)
        self._note_window(full)
        return full

    def _state_bytes(self, n: int) -> int:
        """Algorithmic bytes of the env step itself over n envs (state read + write, small obs,
        lidar, record write, action, reward and flags; config.bytes_per_env_step "state")."""
        from .config import bytes_per_env_step
        return n * bytes_per_env_step(self.cfg, potential=self.potential is not None)["state"]

    def _step_fused(self, actions, timing: Optional[list] = None) -> None:
        """Env step + raster in one launch (ffmp_step_fused): one block per env."""
        self._check_open()
        a = self._actions(actions)
        self._act_keepalive = a
        full = self._next_window()
        flags = self.fused_flags | (0 if full else _abi.RASTER_NEWEST)
        if timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        _abi.check(self.lib.ffmp_step_fused(C.byref(self._cfg_c), self.num_envs, self.env_offset, a.data_ptr(),
                                            C.byref(self._state_c), C.byref(self._obs_c), C.byref(self._out_c), flags,
                                            self._stream()), "ffmp_step_fused")
        if timing is not None:
            e1.record()
            n = self.num_envs
            timing.append((e0, e1, n, self._raster_bytes(n, full) + self._state_bytes(n), full))

    def raster_step(self, timing: Optional[list] = None) -> None:
        """Kernel 2 of a step (the HBM-bound hot kernel): slide the frame pair by one and raster
        the new frame + potential (+ flow), or both frames when the window wraps or W == 2."""
        self._check_open()
        full = self._next_window()
        self._raster_launch(full, None, timing)

    def _step_pipelined(self, actions, timing) -> None:
        self._check_open()
        a = self._actions(actions)
        self._act_keepalive = a
        main = torch.cuda.current_stream(self.device)
        side = self._side
        self._ev_go.record(main)
        side.wait_event(self._ev_go)
        sp = C.c_void_p(side.cuda_stream)
        for k, (a0, n, st, ob, out, rec) in enumerate(self._slices):
            _abi.check(self.lib.ffmp_step_state(C.byref(self._cfg_c), n, self.env_offset + a0,
                                                a.data_ptr() + a0 * 8, C.byref(st), C.byref(ob), C.byref(out), sp),
                       "ffmp_step_state")
            self._ev_slice[k].record(side)
        # the raster of slice k on the main stream once its env slice is done: the env kernels of the
        # later slices run beside it.  The frame pair slides as in raster_step (ring or contiguous).
        full = self._next_window()
        cpb, flags = self.raster_shape if full else self.raster_shape_newest
        flags |= 0 if full else _abi.RASTER_NEWEST
        sm0, sm_stride, sm_frame = self._obs_c.state_m, self._obs_c.state_m_stride, self._obs_c.state_m_frame_stride
        mp = C.c_void_p(main.cuda_stream)
        for k, (a0, n, st, ob, out, rec) in enumerate(self._slices):
            ob.state_m = sm0 + a0 * sm_stride * self._fes
            ob.state_m_stride, ob.state_m_frame_stride = sm_stride, sm_frame
            main.wait_event(self._ev_slice[k])
            if timing is not None:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main)
            _abi.check(self.lib.ffmp_raster_ex(C.byref(self._cfg_c), n, rec, None, C.byref(ob), cpb, flags, mp),
                       "ffmp_raster")
            if timing is not None:
                e1.record(main)
                timing.append((e0, e1, n, self._raster_bytes(n, full), full))

    def step(self, actions, copy: bool = False, timing: Optional[list] = None
             ) -> Tuple[Dict[str, torch.Tensor], torch.Tensor, torch.Tensor, dict]:
        """Advance every env one step. Returns (obs, reward f32[N], done bool[N], info).

        `timing`: optional list; (start, end, n_envs, algorithmic bytes, full) per raster launch
        (HIP events on the caller's stream) are appended to it.  With use_graphs(True) (and no
        `timing`) the step's launches run as the replay of a single-step HIP graph (step_graphs)."""
        self._check_open()
        if self._needs_reset:
            raise RuntimeError("call reset() before step()")
        with torch.cuda.device(self.device):
            if self._graphs is not None and timing is None:
                self._step_graph(actions)
            elif self.pipeline_slices > 1:
                self._step_pipelined(actions, timing)
            elif self.fused:
                self._step_fused(actions, timing)
            else:
                self.step_state(actions)
                self.raster_step(timing)
            self._bev_push(advance=True)
        if self.info_format == "list":
            info = self._info_list()
        else:
            info = {"is_goal": self.is_goal, "collision": self.collision, "truncated": self.truncated,
                    "step": self.t, "episode": self.episode}
            if copy:
                info = {k: v.clone() for k, v in info.items()}
        if copy:
            return self._obs_out(True), self.reward.clone(), self.done.clone(), info
        return self.obs, self.reward, self.done, info

    # ------------------------------------------------ info in gym 0.17/0.18's per-env form
    # "dict" (default): one dict of (N,) device tensors, the batched form (nothing leaves the GPU).
    # "list": gym.vector.VectorEnv.step_wait's form in gym 0.17/0.18 — a tuple of N dicts of Python
    # scalars, one per env (costs one device -> host copy of the five (N,) flags per step).
    info_format = "dict"
    INFO_FORMATS = ("dict", "list")

    def _info_list(self) -> tuple:
        keys = ("is_goal", "collision", "truncated", "t", "episode")  # info key "step" is the counter t
        cols = torch.stack([getattr(self, k).to(torch.int64) for k in keys]).cpu().tolist()
        return tuple({"is_goal": bool(g), "collision": bool(c), "truncated": bool(tr), "step": int(st),
                      "episode": int(ep)} for g, c, tr, st, ep in zip(*cols))

    # ------------------------------------------------ single-step graphs for step()
    # A closed-loop caller (each action computed from the previous observation, train.py:572-577)
    # cannot use capture()'s multi-step graphs.  use_graphs(True): every step() replays a HIP graph of
    # ONE step (its env kernel + raster, or the one-launch step), captured lazily for each frame-ring
    # position (graph_period() of them), reading the actions from a static device buffer
    # (`action_buffer`; step(env.action_buffer) skips the copy into it).  Bit-identical to the plain
    # launches (tests/test_gpu_graph.py).
    _graphs = None

    def use_graphs(self, on: bool = True) -> None:
        """Run step() as single-step graph replays (on) or plain launches (off).  Not with pipeline
        slices or a BEV image ring (their steps need per-step host work)."""
        self._check_open()
        if not on:
            self._graphs = None
            return
        if self.pipeline_slices > 1 or self.bev is not None:
            raise ValueError("use_graphs() needs pipeline=1 and no bev_series")
        if self._graphs is None:
            self._graphs = {}
            if getattr(self, "action_buffer", None) is None:
                self.action_buffer = torch.zeros(self.num_envs, dtype=torch.int64, device=self.device)

    action_buffer = None

    def _step_graph(self, actions) -> None:
        buf = self.action_buffer
        if not (isinstance(actions, torch.Tensor) and actions.data_ptr() == buf.data_ptr()):
            buf.copy_(self._actions(actions), non_blocking=True)
        key = (self._wpos, self.fused)
        g = self._graphs.get(key)
        if g is None:
            g = torch.cuda.CUDAGraph()
            snap = (self._wpos, list(self._hist), self._hist_from_reset)
            stream = torch.cuda.Stream(device=self.device)
            stream.wait_stream(torch.cuda.current_stream(self.device))
            try:
                with torch.cuda.graph(g, stream=stream):
                    if self.fused:
                        self._step_fused(buf)
                    else:
                        self.step_state(buf)
                        self.raster_step()
            finally:
                # nothing ran: the host bookkeeping goes back to where the GPU state is
                self._set_window(snap[0])
                self._hist, self._hist_from_reset = snap[1], snap[2]
            self._graphs[key] = g
        g.replay()
        self._next_window()

    # ------------------------------------------------ closed-loop controller
    def policy_reactive(self, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The next actions (N,) int64 from the current observation, on the device
        (include/ffmp.h ffmp_policy_reactive: steer towards the goal, stop and turn when the newest
        frame is occupied just ahead) — a scripted controller for closed-loop runs (bench.py's
        closed_loop leg), not the reference's Q-network.  `out`: write into this (N,) int64 tensor
        (e.g. action_buffer) instead of a new one."""
        self._check_open()
        if self._needs_reset:
            raise RuntimeError("call reset() before policy_reactive()")
        if out is None:
            out = torch.empty(self.num_envs, dtype=torch.int64, device=self.device)
        elif out.shape != (self.num_envs,) or out.dtype != torch.int64 or not out.is_contiguous() \
                or out.device != self.device:
            raise ValueError(f"out must be a contiguous int64 tensor of shape ({self.num_envs},) on {self.device}")
        with torch.cuda.device(self.device):
            _abi.check(self.lib.ffmp_policy_reactive(C.byref(self._cfg_c), self.num_envs, C.byref(self._obs_c),
                                                     out.data_ptr(), self._stream()), "ffmp_policy_reactive")
        return out

    # ------------------------------------------------ HIP graph of whole steps
    def graph_period(self) -> int:
        """Steps after which the frame pair is back on the same ring slots (so one captured
        sequence of steps can be replayed forever): W with the seamless ring, W - 1 with the
        wrapping ring (its wrap step writes both frames), 1 with W = 2."""
        if self.ring == "seamless":
            return self.frame_window
        return self.frame_window - 1 if self.frame_window > 2 else 1

    def capture(self, steps: Optional[int] = None, pipelined: Optional[bool] = None,
                skewed: Optional[bool] = None, policy=None) -> "StepGraph":
        """Capture `steps` consecutive steps (default graph_period(); a multiple of it) into one HIP
        graph (torch.cuda.CUDAGraph: hipGraph on ROCm).  StepGraph.replay(actions) then runs them as
        ONE launch from the host — every kernel of every step, the same launches step() makes, with
        no host work or launch gaps between them; the actions are read from a static device block the
        replay fills first.  The host's frame bookkeeping is advanced by the replay, not by the
        capture (nothing runs while capturing).  `pipelined` (two-launch steps, an even count; off by
        default, StepGraph.PIPELINE_DEFAULT): the env kernel of step i + 1 runs beside the raster of
        step i (see StepGraph).  `skewed` (float32 frames, no flow planes, the two-launch step, an even
        count; by default where the env step's blocks fit the CUs once, StepGraph._skew_pays): the
        raster of step i and the env step of step i + 1 in ONE launch (ffmp_step_skewed).
        `policy` (closed loop): "reactive" (policy_reactive) or a callable env -> (N,) int64 device
        tensor, captured too: each step's actions are computed inside the graph from the previous
        step's observation (the first from the observation before the replay), and replay() takes
        no actions — the device-resident form of train.py:572-577's act-then-publish loop.  Plain
        two-launch (or one-launch) steps only: the policy reads the raster's frame."""
        return StepGraph(self, steps, pipelined, skewed, policy)

    # ------------------------------------------------ gym.vector.VectorEnv surface
    is_vector_env = True

    @property
    def single_action_space(self):
        """The action id train.py feeds to RobotAction.commander (train.py:343-345, 668-673);
        the reference's Box (ffmp.py:29-32) describes the (v, w) it maps to."""
        from ._spaces import Discrete
        return Discrete(28)

    @property
    def action_space(self):
        from ._spaces import MultiDiscrete
        return MultiDiscrete([28] * self.num_envs)

    def _obs_space(self, lead):
        """Keys/dtypes of the train.py consumer contract (train.py:543-557), bounds per key."""
        from ._spaces import Box, Dict as DictSpace
        G, L = self.cfg.grid, self.cfg.n_beams
        inf = np.inf

        def box(lo, hi, shape, dtype=np.float32):
            lo = np.broadcast_to(np.asarray(lo, dtype=dtype), lead + shape)
            hi = np.broadcast_to(np.asarray(hi, dtype=dtype), lead + shape)
            return Box(lo, hi, dtype=dtype)

        compact = self.obs_format == "u8f16"
        sp = {"state_m": box(0, 255, (2, G, G), np.uint8) if compact else box(0.0, 255.0, (2, G, G)),
              "state_g": box([0.0, -np.pi], [inf, np.pi], (2,)),   # [dist, orient]
              "state_v": box([0.0, -np.pi], [inf, np.pi], (2,)),   # [|dxy|, wrap(dyaw)] per step
              "state_t": box(0.0, inf, (1,)),
              "grad": box(-inf, inf, (2,))}
        if self.potential is not None:
            sp["potential"] = box(0.0, inf, (G, G), np.float16 if compact else np.float32)
        if L:
            sp["lidar"] = box(-inf, inf, (L,))
        if self.flow is not None:
            sp["flow"] = box(-inf, inf, (2, G, G), np.float16 if compact else np.float32)
        return DictSpace(sp)

    @property
    def single_observation_space(self):
        return self._obs_space(())

    @property
    def observation_space(self):
        return self._obs_space((self.num_envs,))

    def seed(self, seed: int) -> None:
        """gym 0.17-style: the seed of the next full reset()."""
        self._set_cfg(self.cfg.replace(seed=int(seed)))

    def _set_cfg(self, cfg: FFMPConfig) -> None:
        """A new config after construction (a new seed): the launch struct is rebuilt, and the
        single-step graphs, which captured the old one by value, are dropped (re-captured on use)."""
        self.cfg = cfg
        self._cfg_c = _abi.make_cfg(self.cfg, _ptr(self.beam_cs) or 0)
        if self._graphs is not None:
            self._graphs = {}

    def step_async(self, actions) -> None:
        self._pending_actions = actions

    def step_wait(self, **kw):
        a, self._pending_actions = self._pending_actions, None
        if a is None:
            raise RuntimeError("step_wait() without step_async()")
        return self.step(a, **kw)

    def close(self) -> None:
        """Release the device buffers (the object is unusable afterwards: every entry point that
        would launch a kernel raises RuntimeError)."""
        if self._closed:
            return
        self._closed = True
        self._needs_reset = True
        torch.cuda.synchronize(self.device)
        self._graphs = None  # their kernels' arguments point into the buffers freed below
        self.action_buffer = None
        for name, _, _ in self._buffer_specs():
            setattr(self, name, None)
        # the launch structs hold raw device pointers into the freed buffers
        self._state_c = self._obs_c = self._out_c = None
        self._slices = []
        self._arena_buf = None
        self._record_alt = None
        self.bev = None
        had_ring = self.ring == "seamless"
        self._ring = None  # the seamless ring's pieces return to the process pool ...
        self._forget_partners()  # the potential plane is freed: its pairing references go
        torch.cuda.empty_cache()
        if had_ring and self.release_pool:
            import gc
            gc.collect()  # ... once the last tensor view of the ring is gone
            _abi.ring_pool_trim(self.device.index, self.pool_keep_bytes)  # ... and their memory to the device

    _closed = False
    bev = None  # the BEV image ring (bev_series); a class default: _alloc's HBM accounting runs first

    def _check_open(self) -> None:
        if self._closed:
            raise RuntimeError("FFMPVec is closed")

    # ------------------------------------------------------------ utilities
    def check_errors(self) -> None:
        """Raise if any step saw an action id outside 0..27 (it was run as action 3)."""
        v = int(self.err.item())
        if v:
            self.err.zero_()
            raise ValueError(f"invalid action id(s) passed to FFMPVec.step (error bits {v:#x})")

    # simulator state, then the per-env observations and outputs the env kernel wrote (the planes
    # are re-rastered from the record on load)
    _SD_STATE = ("pose", "goal", "d0", "obst", "obst_r", "t", "episode", "record")
    _SD_OBS = ("state_g", "state_v", "state_t", "grad", "lidar", "reward", "done", "is_goal", "collision",
               "truncated", "term_record", "term_obs")

    def state_dict(self) -> Dict[str, torch.Tensor]:
        """Checkpoint: the simulator state plus the small observations and step outputs (the
        planes are re-derived from the record by load_state_dict's raster())."""
        self._check_open()
        sd = {k: getattr(self, k).clone() for k in self._SD_STATE}
        for k in self._SD_OBS:
            v = getattr(self, k)
            if v is not None:
                sd[k] = v.clone()
        sd["seed"] = torch.tensor(self.cfg.seed, dtype=torch.int64)
        return sd

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        """Restore a state_dict() of an env of the same config and num_envs (a fresh instance
        included): every observation key of the saved env is reproduced."""
        self._check_open()
        for k in self._SD_STATE:
            getattr(self, k).copy_(sd[k])
        for k in self._SD_OBS:
            v = getattr(self, k)
            if v is not None and k in sd:
                v.copy_(sd[k])
        seed = int(sd["seed"])
        if seed != self.cfg.seed:
            self._set_cfg(self.cfg.replace(seed=seed))
        self.raster()
        self._hist, self._hist_from_reset = [], False  # older frames than the pair are not restored
        self._note_window(True)
        self._bev_hist, self._bev_from_reset = [self._bev_pos], False  # likewise older BEV images
        self._needs_reset = False

    def hbm_bytes(self) -> int:
        """HBM this instance holds now: its arena plus the seamless ring's W physical slots (the
        alias slot maps slot 0's pages again and holds nothing)."""
        ring = 0
        if self.ring == "seamless" and getattr(self, "_ring", None) is not None:
            ring = self.frame_window * self._ring.slot_stride
        alt = getattr(self, "_record_alt", None)  # a pipelined step graph's second record buffer
        if self._arena_buf is not None:
            return self._arena_buf.numel() + ring + (0 if alt is None else alt.numel() * alt.element_size())
        return ring + sum(t.numel() * t.element_size() for t in vars(self).values()
                          if isinstance(t, torch.Tensor) and not (ring and t is self.frames))

    def __repr__(self):
        c = self.cfg
        return (f"FFMPVec(num_envs={self.num_envs}, G={c.grid}, K={c.n_obst}, L={c.n_beams}, "
                f"moving={c.moving}, device={self.device}, env_offset={self.env_offset}, "
                f"frame_window={self.frame_window}, ring={self.ring}, obs_format={self.obs_format})")


__all__ = ["FFMPVec", "PRESETS"]


class StepGraph:
    """`steps` consecutive FFMPVec steps captured as one HIP graph (FFMPVec.capture).

    The env kernel + raster (or the one-launch step) of each step are recorded with the frame-ring
    slots that step writes; when `steps` is a multiple of graph_period() the ring is back on its
    starting slots after a replay and the same graph is valid for the next one (other counts replay
    whenever the frame position is back where the capture started).  replay(actions)
    copies the (steps, N) action block into the graph's static block (one device copy), replays,
    then advances the env's host-side frame bookkeeping exactly as `steps` calls of step() would.
    Results are those of `steps` step() calls with the same actions, bit for bit
    (tests/test_gpu_graph.py).  Not with pipeline slices or a BEV image ring (their launches need
    per-step host work), and the env must not be stepped or reset between capture and replay except
    through whole replays or whole periods of step() calls (checked: the frame position).

    Pipelined (two-launch steps, an even step count): the raster of step i reads only the record
    its env kernel wrote, and the env kernel reads none of the raster's outputs, so with two record
    buffers — step i's env kernel writes buffer (i + 1) % 2, the current record being buffer 0 —
    the env kernel of step i + 1 runs on a second stream beside the raster of step i, waiting only
    for the raster of step i - 1 (the last reader of its buffer).  The graph's intermediate steps'
    small outputs (reward, done, state_g, ...) are overwritten one step early, which nobody sees: a
    replay's observation is its last step's, written in the same order as step() writes it, and the
    frames, potential and record are bit-identical (tests/test_gpu_graph.py).

    Skewed (the default where skew_supported() and the one-off trial in _skew_pays() say it pays):
    the same two record buffers, but the raster of step i and the env kernel of step i + 1 are ONE
    launch (ffmp_step_skewed: env blocks first, raster blocks after), so a k-step replay is k + 1
    dispatches on one stream instead of 2k and no env kernel waits on a raster tail.  Same results,
    bit for bit (tests/test_gpu_graph.py, tests/timed_path_check.py)."""

    # Off by default: the overlap happens (rocprofv3 trace, profiles/r05n_pipelined_graph.txt) but the
    # raster beside an env kernel runs ~12 % longer and the graph leaves ~10 us between two rasters on
    # different queues — C2 38.5-38.7 vs 38.9-39.2 M serial, C3 14.01-14.03 vs 13.88-14.03 M
    # (profiles/r05m_pipelined_graph.txt).  FFMP_GRAPH_PIPELINE=1 makes it the default.
    PIPELINE_DEFAULT = os.environ.get("FFMP_GRAPH_PIPELINE", "0") == "1"
    SKEW_DEFAULT = os.environ.get("FFMP_GRAPH_SKEW", "1") != "0"  # A/B knob

    @staticmethod
    def skew_supported(env: FFMPVec, k: int) -> bool:
        """Does ffmp_step_skewed take this instance's steps?  The library answers
        (ffmp_step_skewed_check: float32 frames, no flow planes, its env waves' LDS against the
        device's limit) for both raster shapes the graph uses; the two-launch step and an even k."""
        if env.fused or k % 2 or env.obs_format != "f32" or env.flow is not None:
            return False
        return all(env.lib.ffmp_step_skewed_check(C.byref(env._cfg_c), env._fmt, flags) == 0
                   for flags in {env.raster_shape[1], env.raster_shape_newest[1]})

    @staticmethod
    def _skew_pays(env: FFMPVec) -> bool:
        """The default: skew while the env step's blocks (4 waves each) fit the CUs once — they are
        dispatched first, and more of them delay the raster's stores (C2's 128 blocks: 39.6 -> 41.2 M
        env-steps/s; C3's 2,048: 14.0 -> 13.9 M; profiles/r05r_skewed_graph.txt).  bench.py times both."""
        K = env.cfg.n_obst
        lpe = 8 if K <= 8 else 16 if K <= 16 else 32 if K <= 32 else 64
        blocks = -(-env.num_envs // (4 * (64 // lpe)))
        return blocks <= torch.cuda.get_device_properties(env.device).multi_processor_count

    def __init__(self, env: FFMPVec, steps: Optional[int] = None, pipelined: Optional[bool] = None,
                 skewed: Optional[bool] = None, policy=None):
        env._check_open()
        if policy is not None:
            if pipelined or skewed:
                raise ValueError("a closed-loop graph (policy) runs plain steps: the policy reads each raster's frame")
            if policy != "reactive" and not callable(policy):
                raise ValueError("policy must be 'reactive' or a callable env -> (N,) int64 tensor")
            pipelined = skewed = False
        self.policy = policy
        if env._needs_reset:
            raise RuntimeError("call reset() before capture()")
        if env.pipeline_slices > 1 or env.bev is not None:
            raise ValueError("capture() needs pipeline=1 and no bev_series")
        per = env.graph_period()
        k = per if steps is None else int(steps)
        if k <= 0:
            raise ValueError("steps must be positive")
        # a multiple of the period ends on the slots it started from, so it replays back to back;
        # any other count is replayable once the frame position is back at the capture's
        self.chainable = k % per == 0
        self.env, self.steps = env, k
        self.actions = torch.zeros((k, env.num_envs), dtype=torch.int64, device=env.device)
        can_pipe = not env.fused and k % 2 == 0
        if pipelined is None:
            pipelined = can_pipe and self.PIPELINE_DEFAULT
        if pipelined and not can_pipe:
            raise ValueError("a pipelined graph needs the two-launch step and an even step count")
        self.pipelined = bool(pipelined)
        can_skew = not self.pipelined and self.skew_supported(env, k)
        if skewed is None:
            skewed = can_skew and self.SKEW_DEFAULT and self._skew_pays(env)
        if skewed and not can_skew:
            raise ValueError("a skewed graph needs the two-launch step, an even step count, float32 frames "
                             "without flow planes, and no pipelining")
        self.skewed = bool(skewed)
        snap = (env._wpos, list(env._hist), env._hist_from_reset)
        self.wpos = env._wpos
        self.graph = torch.cuda.CUDAGraph()
        stream = torch.cuda.Stream(device=env.device)
        torch.cuda.synchronize(env.device)
        rec0 = env.record
        if self.pipelined or self.skewed:
            if getattr(env, "_record_alt", None) is None or env._record_alt.shape != rec0.shape:
                env._record_alt = torch.empty_like(rec0)
            bufs = (rec0, env._record_alt)
        if self.pipelined:
            self._side = torch.cuda.Stream(device=env.device)
        try:
            with torch.cuda.device(env.device), torch.cuda.graph(self.graph, stream=stream):
                if self.pipelined:
                    self._capture_pipelined(k, bufs)
                elif self.skewed:
                    self._capture_skewed(k, bufs)
                else:
                    for i in range(k):
                        if policy is not None:
                            self._act(i)
                        if env.fused:
                            env._step_fused(self.actions[i])
                        else:
                            env.step_state(self.actions[i])
                            env.raster_step()
        finally:
            env.record = rec0
            env._state_c.record = rec0.data_ptr()
            # nothing ran: the host bookkeeping goes back to where the GPU state is
            env._set_window(snap[0])
            env._hist, env._hist_from_reset = snap[1], snap[2]
        if env._wpos != self.wpos:
            raise RuntimeError("frame position changed during capture")

    def _act(self, i: int) -> None:
        """Closed loop: step i's actions from the current observation, into the static block."""
        if self.policy == "reactive":
            self.env.policy_reactive(out=self.actions[i])
        else:
            a = self.policy(self.env)
            if not (isinstance(a, torch.Tensor) and a.numel() == self.env.num_envs):
                raise ValueError("policy must return an (N,) tensor of action ids")
            self.actions[i].copy_(a.reshape(-1))

    def _capture_pipelined(self, k: int, bufs) -> None:
        env, side = self.env, self._side
        cap = torch.cuda.current_stream(env.device)
        fork = torch.cuda.Event()
        fork.record(cap)
        side.wait_event(fork)
        ev_env = [torch.cuda.Event() for _ in range(k)]
        ev_ras = [torch.cuda.Event() for _ in range(k)]
        for i in range(k):
            buf = bufs[(i + 1) % 2]  # k even: the last step writes buffer 0, the current record
            env.record = buf
            env._state_c.record = buf.data_ptr()
            with torch.cuda.stream(side):
                if i >= 2:
                    side.wait_event(ev_ras[i - 2])  # the last raster that read this buffer
                env.step_state(self.actions[i])
                ev_env[i].record(side)
            cap.wait_event(ev_env[i])
            env.raster_step()
            ev_ras[i].record(cap)
        # the side stream's last work (env kernel k - 1) is joined by the last raster's wait

    def _capture_skewed(self, k: int, bufs) -> None:
        """env(0); then for i < k - 1 ONE launch of raster(i) + env(i + 1); then raster(k - 1).  env(i)
        writes record buffer (i + 1) % 2, raster(i) reads it (k even: the last is buffer 0)."""
        env = self.env
        env.record = bufs[1]
        env._state_c.record = bufs[1].data_ptr()
        env.step_state(self.actions[0])
        for i in range(k - 1):
            full = env._next_window()
            cpb, flags = env.raster_shape if full else env.raster_shape_newest
            flags |= 0 if full else _abi.RASTER_NEWEST
            rec_r, rec_w = bufs[(i + 1) % 2], bufs[(i + 2) % 2]
            env.record = rec_w
            env._state_c.record = rec_w.data_ptr()
            _abi.check(env.lib.ffmp_step_skewed(C.byref(env._cfg_c), env.num_envs, env.env_offset,
                                                self.actions[i + 1].data_ptr(), C.byref(env._state_c),
                                                C.byref(env._obs_c), C.byref(env._out_c), rec_r.data_ptr(), cpb,
                                                flags, env._stream()), "ffmp_step_skewed")
        env.record = bufs[0]
        env._state_c.record = bufs[0].data_ptr()
        env.raster_step()

    def replay(self, actions: Optional[torch.Tensor] = None) -> None:
        """Run the captured steps; actions (steps, N) int64 (None: the block the last replay used)."""
        env = self.env
        env._check_open()
        if env._needs_reset:
            raise RuntimeError("call reset() before replay()")
        if env._wpos != self.wpos:
            raise RuntimeError("the env's frame position moved since capture (step() a whole graph_period())")
        if actions is not None:
            if self.policy is not None:
                raise ValueError("a closed-loop graph computes its own actions (replay() takes none)")
            a = torch.as_tensor(actions)
            if a.shape != self.actions.shape:
                raise ValueError(f"actions must have shape {tuple(self.actions.shape)}")
            self.actions.copy_(a, non_blocking=True)
        with torch.cuda.device(env.device):
            self.graph.replay()
        for _ in range(self.steps):  # the host side of each step (frame pair, history), no launch
            env._next_window()
