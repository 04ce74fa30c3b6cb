"""ReplayMemory — a device-resident transition store for FFMPVec.

The reference keeps a Python list of `Transition` namedtuples (src/train.py:44, 212-228),
each holding two float32 (1,2,100,100) map stacks, and concatenates a minibatch on the host
for every update (`Brain.make_minibatch`, :352-372).  Batched on one GPU that is ~1 MB per
transition at 256² and a host round trip per sample.

Here a transition is stored as what GENERATES its observations: the raster record of the
state (the env's record before the step) and of the observation (its post-step record before
auto-reset, `keep_terminal=True`), plus the small obs, action, reward and done —
2 x (16 + 12K) + 10 floats + 13 B (1,717 B at C3, ~600x smaller than two f32 map stacks).
`sample(B)` gathers B records of each kind and re-runs the raster kernel on them, producing
the minibatch tensors in the reference's layout directly in HBM: bit-identical to the
state_m / observe_m the env emitted (the raster is a pure function of the record).

  ReplayMemory.push (:218-222)  -> push_begin(env) before env.step + push_end(env, action) after:
                                   N transitions at slots index .. index+N-1 (mod capacity)
  ReplayMemory.sample (:224-225) -> sample(B): uniform without replacement, like random.sample
  ReplayMemory.__len__ (:227-228) -> len()
  Brain.make_minibatch (:352-372) -> the returned Transition of batched tensors

Transitions are causal: (obs_t, a_t, obs_t+1, r_t+1).  (The reference's asynchronous ROS loop
pairs the action chosen from obs_t-1 with obs_t; a synchronous env has no such skew.)

series=k > 2 (make_temporal_maps over k mono frames, train.py:66-69, 474-486; FFMPVec.temporal_maps):
a transition also keeps the records of the k-2 steps before its state and the state's steps since
reset; sample() rasters the k frames of each side, the lag-d frame being the newest frame of the
record d steps back, clamped to the episode start (the last frame is the older frame of the record
k-2 steps back: k-1 raster launches write k frames per sample).  The memory keeps the k-2 previous
records of every env itself (push_begin must see every step); a transition pushed less than k-2
steps after the memory was created sees its deepest lags clamped to the oldest record it has.

bev=True (the 12-channel option, train.py:66: "(occupancy(MONO) + flow(RGB)) * series(3 steps)";
FFMPVec(bev_series=k).bev_maps): the maps are k 4-channel BEV images [occupancy, R, G, B], oldest
first (include/ffmp.h ffmp_bev_image).  The lag-d image needs the flow of the record d steps back,
so a transition keeps the k-1 records before its state; sample() rasters each lag's record (newest
frame + flow planes) and colours it into its 4 channels: 2k raster + 2k colour launches per batch.
"""
from __future__ import annotations

import ctypes as C
from collections import namedtuple
from typing import Optional, Tuple

import numpy as np
import torch

from . import _abi

# Field order of the reference's Transition (train.py:44)
Transition = namedtuple("Transition", ("state_m", "state_g", "state_v", "state_t", "action", "observe_m",
                                       "observe_g", "observe_v", "observe_t", "reward"))


class ReplayMemory:
    """Ring buffer of `capacity` transitions of `env` (an FFMPVec built with keep_terminal=True).

    sample() materialises the map stacks with the env's raster kernel (state_m / observe_m
    f32 (B,2,G,G); with `potential=True` also the potential planes (B,G,G) of both sides)."""

    def __init__(self, env, capacity: int, seed: int = 0, series: int = 2, bev: bool = False):
        if not getattr(env, "keep_terminal", False):
            raise ValueError("ReplayMemory needs FFMPVec(..., keep_terminal=True) (terminal records of done envs)")
        if capacity < env.num_envs:
            raise ValueError(f"capacity {capacity} < num_envs {env.num_envs}: one step would overwrite itself")
        self.env, self.cfg, self.lib = env, env.cfg, env.lib
        self.capacity = int(capacity)
        self.device = env.device
        R, dev = self.cfg.record_len(), self.device
        self.s_record = torch.zeros(self.capacity, R, dtype=torch.float32, device=dev)
        self.o_record = torch.zeros(self.capacity, R, dtype=torch.float32, device=dev)
        self.s_small = torch.zeros(self.capacity, 5, dtype=torch.float32, device=dev)  # g[2], v[2], t
        self.o_small = torch.zeros(self.capacity, 5, dtype=torch.float32, device=dev)
        self.action = torch.zeros(self.capacity, dtype=torch.int64, device=dev)
        self.reward = torch.zeros(self.capacity, dtype=torch.float32, device=dev)
        self.done = torch.zeros(self.capacity, dtype=torch.bool, device=dev)
        self.series = int(series)
        if not 1 <= self.series <= _abi.MAX_SERIES:
            raise ValueError(f"series must be in [1, {_abi.MAX_SERIES}]")
        self.bev = bool(bev)
        if self.bev and not self.cfg.flow:
            raise ValueError("bev=True needs an env with FFMPConfig(flow=True)")
        # the mono series' oldest frame is the older frame of record r_t-k+2; a BEV image needs
        # that record's own flow, so one more record back
        H = self.series - 1 if self.bev else max(self.series - 2, 0)
        self._H = H
        # series > 2: records r_t-1 .. r_t-k+2 of the state, its steps since reset, and every env's
        # last k-2 records (newest first; `_seen` steps of them are real)
        self.s_hist = torch.zeros(self.capacity, H, R, dtype=torch.float32, device=dev) if H else None
        self.s_since = torch.zeros(self.capacity, dtype=torch.int32, device=dev) if H else None
        self._env_hist = torch.zeros(H, env.num_envs, R, dtype=torch.float32, device=dev) if H else None
        self._seen = 0
        self.index = 0   # next slot (train.py:216)
        self.size = 0    # len(self.memory)
        self._pending = None
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(int(seed))
        self._cfg_c = _abi.make_cfg(self.cfg, env.beam_cs.data_ptr() if env.beam_cs is not None else 0)
        self._bufs = {}

    def __len__(self) -> int:
        return self.size

    def _tensors(self):
        return [t for t in (self.s_record, self.o_record, self.s_small, self.o_small, self.action, self.reward,
                            self.done, self.s_hist, self.s_since, self._env_hist) if t is not None]

    def hbm_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self._tensors())

    # ----------------------------------------------------------------- push
    def _slots(self, n: int):
        a = self.index
        first = min(n, self.capacity - a)
        return [(a, 0, first)] + ([(0, first, n - first)] if first < n else [])

    def push_begin(self, env=None) -> None:
        """Before env.step(): record the current observation of every env as the transitions'
        state (its raster record + state_g/state_v/state_t)."""
        env = env or self.env
        n = env.num_envs
        small = torch.cat([env.state_g, env.state_v, env.state_t], dim=1)
        H = self._H
        if H > 0:
            since = env.t.clamp(max=self._seen)
        for dst, src, cnt in self._slots(n):
            self.s_record[dst:dst + cnt].copy_(env.record[src:src + cnt])
            self.s_small[dst:dst + cnt].copy_(small[src:src + cnt])
            if H > 0:
                self.s_hist[dst:dst + cnt].copy_(self._env_hist[:, src:src + cnt].transpose(0, 1))
                self.s_since[dst:dst + cnt].copy_(since[src:src + cnt])
        if H > 0:  # the next step's history: this state's record first
            self._env_hist.copy_(torch.cat((env.record.unsqueeze(0), self._env_hist[:H - 1])))
            self._seen = min(self._seen + 1, H)
        self._pending = n

    def push_end(self, action: torch.Tensor, env=None) -> None:
        """After env.step(action): the observation (terminal state for envs that reset), action,
        reward and done complete the N transitions; the ring index advances by N."""
        env = env or self.env
        n = env.num_envs
        if self._pending != n:
            raise RuntimeError("push_end() without a matching push_begin()")
        action = torch.as_tensor(action, device=self.device).reshape(n).to(torch.int64)
        for dst, src, cnt in self._slots(n):
            self.o_record[dst:dst + cnt].copy_(env.term_record[src:src + cnt])
            self.o_small[dst:dst + cnt].copy_(env.term_obs[src:src + cnt])
            self.action[dst:dst + cnt].copy_(action[src:src + cnt])
            self.reward[dst:dst + cnt].copy_(env.reward[src:src + cnt])
            self.done[dst:dst + cnt].copy_(env.done[src:src + cnt])
        self.index = (self.index + n) % self.capacity
        self.size = min(self.size + n, self.capacity)
        self._pending = None

    # --------------------------------------------------------------- sample
    def _batch_planes(self, key: str, B: int, potential: bool):
        G = self.cfg.grid
        want = (B, potential)
        if self._bufs.get(key, (None,))[0] != want:
            sm = torch.empty(B, max(self.series, 2), G, G, dtype=torch.float32, device=self.device)
            pot = torch.empty(B, G, G, dtype=torch.float32, device=self.device) if potential else None
            flow = torch.empty(B, 2, G, G, dtype=torch.float32, device=self.device) if self.cfg.flow else None
            self._bufs[key] = (want, sm, pot, flow)
        return self._bufs[key][1:]

    def _raster(self, records: torch.Tensor, sm, pot, flow, pos: int = 0, newest_only: bool = False) -> None:
        """Raster `records` into sm[:, pos] (older) and sm[:, pos + 1] (newest); newest_only: the
        older frame only for reset records (FFMP_RASTER_NEWEST)."""
        G2 = self.cfg.grid * self.cfg.grid
        ob = _abi.ObsT(sm.data_ptr() + pos * G2 * sm.element_size(), None, None, None,
                       pot.data_ptr() if pot is not None else None, None, None,
                       flow.data_ptr() if flow is not None else None)
        ob.state_m_stride, ob.state_m_frame_stride = sm.shape[1] * G2, G2
        cpb, flags = self.env.raster_shape
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        with torch.cuda.device(self.device):
            _abi.check(self.lib.ffmp_raster_ex(C.byref(self._cfg_c), records.shape[0], records.data_ptr(), None,
                                               C.byref(ob), cpb, flags | (_abi.RASTER_NEWEST if newest_only else 0),
                                               stream), "ffmp_raster")

    def _raster_series(self, recs: torch.Tensor, since: torch.Tensor, sm, pot, flow) -> None:
        """k frames per sample from recs (B, k-1, R) = records r_t, r_t-1, ..., r_t-k+2: the lag-d
        frame (d <= k-2) is the newest frame of r_t-min(d, since), the lag-(k-1) frame the older
        frame of r_t-min(k-2, since) (a reset record's older frame is its newest).  Frames two
        launches both write carry the same values."""
        k = self.series
        B = recs.shape[0]
        ar = torch.arange(B, device=self.device)
        for d in range(k - 1):
            j = since.to(torch.int64).clamp(max=d)
            rec = recs[ar, j].contiguous()
            full = d == k - 2
            # the potential / flow planes belong to the newest frame only (d = 0)
            self._raster(rec, sm, pot if d == 0 else None, flow if d == 0 else None, pos=k - 2 - d,
                         newest_only=not full)

    def _bev_planes(self, key: str, B: int, potential: bool):
        G, k = self.cfg.grid, self.series
        want = (B, potential)
        if self._bufs.get(key, (None,))[0] != want:
            out = torch.empty(B, 4 * k, G, G, dtype=torch.float32, device=self.device)
            sm = torch.empty(B, 2, G, G, dtype=torch.float32, device=self.device)
            flow = torch.empty(B, 2, G, G, dtype=torch.float32, device=self.device)
            pot = torch.empty(B, G, G, dtype=torch.float32, device=self.device) if potential else None
            self._bufs[key] = (want, out, sm, flow, pot)
        return self._bufs[key][1:]

    def _bev_series(self, recs: torch.Tensor, since: torch.Tensor, out, sm, flow, pot) -> None:
        """k BEV images per sample from recs (B, k, R) = records r_t, ..., r_t-k+1: the lag-d image
        is [newest frame, flow colours] of r_t-min(d, since), written to channels 4(k-1-d) .."""
        k, G2 = self.series, self.cfg.grid * self.cfg.grid
        B = recs.shape[0]
        ar = torch.arange(B, device=self.device)
        vmax = float(np.float32(self.cfg.obst_vmax))
        stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        # the compact env colours its binary16 flow planes (ffmp_bev_image compact=1): round the
        # re-rastered float32 flow the same way (nearest even), so the learner replays exactly the
        # images it acted on
        compact = getattr(self.env, "obs_format", "f32") == "u8f16"
        for d in range(k):
            j = since.to(torch.int64).clamp(max=d)
            rec = recs[ar, j].contiguous()
            self._raster(rec, sm, pot if d == 0 else None, flow, newest_only=True)
            if compact:
                flow.copy_(flow.to(torch.float16))
            dst = out.data_ptr() + 4 * (k - 1 - d) * G2 * out.element_size()
            with torch.cuda.device(self.device):
                _abi.check(self.lib.ffmp_bev_image(B, 0, sm[:, 1].data_ptr(), 2 * G2, flow.data_ptr(), G2, vmax, dst,
                                                   4 * k * G2, stream), "ffmp_bev_image")

    def sample_indices(self, batch_size: int, replacement: bool = False) -> torch.Tensor:
        if batch_size > self.size and not replacement:
            raise ValueError(f"sample larger than population ({batch_size} > {self.size})")  # as random.sample
        if replacement:
            return torch.randint(0, self.size, (batch_size,), generator=self.gen, device=self.device)
        return torch.randperm(self.size, generator=self.gen, device=self.device)[:batch_size]

    def sample(self, batch_size: int, replacement: bool = False, potential: bool = False,
               index: Optional[torch.Tensor] = None) -> Tuple[Transition, dict]:
        """A minibatch (Brain.make_minibatch layout) and extras {done, index[, potential,
        observe_potential, flow, observe_flow]}.  The returned planes are reused by the next
        sample() call of the same batch size (clone to keep them)."""
        idx = self.sample_indices(batch_size, replacement) if index is None else index.to(self.device)
        B = idx.numel()
        s_rec = self.s_record.index_select(0, idx)
        o_rec = self.o_record.index_select(0, idx)
        if self.bev:
            s_out, s_tmp, s_flow, s_pot = self._bev_planes("bs", B, potential)
            o_out, o_tmp, o_flow, o_pot = self._bev_planes("bo", B, potential)
            s_since = self.s_since.index_select(0, idx) if self._H else torch.zeros(B, dtype=torch.int32,
                                                                                    device=self.device)
            parts = [s_rec.unsqueeze(1)] + ([self.s_hist.index_select(0, idx)] if self._H else [])
            s_recs = torch.cat(parts, 1)                                                 # r_t .. r_t-k+1
            o_recs = torch.cat((o_rec.unsqueeze(1), s_recs[:, :self.series - 1]), 1)     # r_t+1 .. r_t-k+2
            self._bev_series(s_recs, s_since, s_out, s_tmp, s_flow, s_pot)
            self._bev_series(o_recs, s_since + 1, o_out, o_tmp, o_flow, o_pot)
            s_sm, o_sm = s_out, o_out
        else:
            s_sm, o_sm = self._sample_mono(idx, s_rec, o_rec, potential)
            s_pot, o_pot = self._last_pot
        ss = self.s_small.index_select(0, idx)
        os_ = self.o_small.index_select(0, idx)
        tr = Transition(s_sm, ss[:, 0:2], ss[:, 2:4], ss[:, 4:5], self.action.index_select(0, idx).view(B, 1),
                        o_sm, os_[:, 0:2], os_[:, 2:4], os_[:, 4:5], self.reward.index_select(0, idx))
        extra = {"done": self.done.index_select(0, idx), "index": idx}
        if potential:
            extra["potential"], extra["observe_potential"] = s_pot, o_pot
        if self.cfg.flow and not self.bev:
            extra["flow"], extra["observe_flow"] = self._last_flow
        return tr, extra

    def _sample_mono(self, idx, s_rec, o_rec, potential: bool):
        """state_m / observe_m of the mono-frame series (k frames, or the [older, newest] pair)."""
        B = idx.numel()
        s_sm, s_pot, s_flow = self._batch_planes("s", B, potential)
        o_sm, o_pot, o_flow = self._batch_planes("o", B, potential)
        if self.series > 2:
            hist = self.s_hist.index_select(0, idx)
            s_since = self.s_since.index_select(0, idx)
            s_recs = torch.cat((s_rec.unsqueeze(1), hist), 1)                          # r_t .. r_t-k+2
            o_recs = torch.cat((o_rec.unsqueeze(1), s_rec.unsqueeze(1), hist[:, :-1]), 1)  # r_t+1 .. r_t-k+3
            self._raster_series(s_recs, s_since, s_sm, s_pot, s_flow)
            self._raster_series(o_recs, s_since + 1, o_sm, o_pot, o_flow)
        else:
            self._raster(s_rec, s_sm, s_pot, s_flow)
            self._raster(o_rec, o_sm, o_pot, o_flow)
            if self.series == 1:  # the newest frame only (a view)
                s_sm, o_sm = s_sm[:, 1:], o_sm[:, 1:]
        self._last_pot, self._last_flow = (s_pot, o_pot), (s_flow, o_flow)
        return s_sm, o_sm

    _SD = ("s_record", "o_record", "s_small", "o_small", "action", "reward", "done", "s_hist", "s_since", "_env_hist")

    def state_dict(self) -> dict:
        sd = {k: getattr(self, k).clone() for k in self._SD if getattr(self, k) is not None}
        sd.update(index=self.index, size=self.size, series=self.series, seen=self._seen, bev=self.bev)
        return sd

    def load_state_dict(self, sd: dict) -> None:
        if int(sd.get("series", 2)) != self.series or bool(sd.get("bev", False)) != self.bev:
            raise ValueError(f"state_dict of a series={sd.get('series', 2)} bev={sd.get('bev', False)} memory, "
                             f"this one has series={self.series} bev={self.bev}")
        for k in self._SD:
            if getattr(self, k) is not None:
                getattr(self, k).copy_(sd[k])
        self.index, self.size, self._seen = int(sd["index"]), int(sd["size"]), int(sd.get("seen", 0))
