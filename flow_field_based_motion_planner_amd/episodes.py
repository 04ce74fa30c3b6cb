"""EpisodeTracker — the training loop's episode bookkeeping, batched and resident in HBM.

The reference keeps these counters as Python locals of its main loop (src/train.py):

    episode, step, total_step, reach_times, is_first    :501-505   -> init()
    reach_times.append(is_goal); window of 10; average  :579-587   -> reach_rate (float64)
    is_first = False                                    :593
    if step == MAX_STEPS: is_done = True                :607       -> max_steps (0: env already truncates)
    if is_done: episode += 1; step = 0; ...             :611-662
        if reach_rate > REACH_RATE_THRESHOLD: complete  :644       (only once `brain.loss` exists: `armed`)
    else: step += 1; total_step += 1                    :681-682

Here one record per env is updated by one HIP kernel per step (ffmp_episode_update,
include/ffmp.h), fed by an env's flag tensors; running totals over all envs are kept on the
device so logging needs one 64-byte copy instead of per-env reductions.  The reference's quirks
are kept: the reach window counts steps rather than episodes, and the step that ends an
episode does not count towards total_step.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional

import torch

from . import _abi

TOTAL_KEYS = ("env_steps", "episodes", "goals", "collisions", "truncations", "completions", "counted_steps")


class EpisodeTracker:
    """Per-env episode / reach-rate bookkeeping for `num_envs` envs on one GPU.

    Args:
        num_envs: envs tracked (same order as the env's flag tensors).
        window: REACH_MEMORY_CAPACITY (train.py:76), 1..64.
        threshold: REACH_RATE_THRESHOLD (train.py:75).
        max_steps: apply train.py:607 here as well; 0 (default) when the env's done
            flag already includes truncation (FFMPVec does, at t == max_steps).
        armed: the reference only runs the completion test once a loss exists
            (train.py:620); set False until the learner has produced one.
        reset_iteration: also run the loop's reset-observation iteration (the is_first
            iteration that observes a freshly reset world, train.py:532-566) at start and after
            every done, which a batched env folds into the resetting step.  True (default)
            makes every counter equal the reference loop's for the same episodes; then
            `step == env.t + 1`.  False counts env steps only (`step == env.t`).
    """

    def __init__(self, num_envs: int, window: int = 10, threshold: float = 0.80, max_steps: int = 0,
                 armed: bool = True, reset_iteration: bool = True, device: Optional[torch.device] = None):
        if not 1 <= int(window) <= 64:
            raise ValueError(f"window must be in [1, 64], got {window}")
        if num_envs < 0 or max_steps < 0:
            raise ValueError("num_envs and max_steps must be >= 0")
        self.lib = _abi.load()
        self.num_envs, self.window, self.threshold = int(num_envs), int(window), float(threshold)
        self.max_steps, self.armed, self.reset_iteration = int(max_steps), bool(armed), bool(reset_iteration)
        self.device = torch.device(device if device is not None else torch.cuda.current_device())
        if self.device.type != "cuda":
            raise _abi.FFMPBackendError("EpisodeTracker needs a GPU device (no CPU path)")
        n, dev = self.num_envs, self.device
        self.reach_bits = torch.zeros(n, dtype=torch.int64, device=dev)
        self.reach_len = torch.zeros(n, dtype=torch.int32, device=dev)
        self.reach_rate = torch.zeros(n, dtype=torch.float64, device=dev)
        self.step = torch.zeros(n, dtype=torch.int32, device=dev)
        self.episode = torch.zeros(n, dtype=torch.int32, device=dev)
        self.total_step = torch.zeros(n, dtype=torch.int64, device=dev)
        self.is_first = torch.ones(n, dtype=torch.bool, device=dev)
        self.complete = torch.zeros(n, dtype=torch.bool, device=dev)
        self.totals = torch.zeros(_abi.EP_TOTALS, dtype=torch.int64, device=dev)
        self._ep_c = _abi.EpisodeT(*(t.data_ptr() for t in (
            self.reach_bits, self.reach_len, self.reach_rate, self.step, self.episode, self.total_step,
            self.is_first, self.complete, self.totals)))
        self.init()

    def _flags(self) -> int:
        return (_abi.EP_ARMED if self.armed else 0) | (_abi.EP_RESET_ITER if self.reset_iteration else 0)

    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def init(self, mask: Optional[torch.Tensor] = None) -> None:
        """Loop start values (train.py:501-505) for the masked envs (all, and totals, if None),
        followed by the reset-observation iteration when `reset_iteration`."""
        mp = None
        if mask is not None:
            mask = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            if mask.numel() != self.num_envs:
                raise ValueError("mask must have num_envs elements")
            mp = mask.data_ptr()
        with torch.cuda.device(self.device):
            _abi.check(self.lib.ffmp_episode_init(self.num_envs, mp, self._flags(), C.byref(self._ep_c),
                                                  self._stream()), "ffmp_episode_init")

    def update(self, done: torch.Tensor, is_goal: torch.Tensor, collision: Optional[torch.Tensor] = None,
               truncated: Optional[torch.Tensor] = None) -> None:
        """One loop iteration from a step's (N,) flag tensors (bool or uint8, on this device)."""
        def flag(t, name):
            if t is None:
                t = torch.zeros(self.num_envs, dtype=torch.uint8, device=self.device)
            if t.device != self.device or t.numel() != self.num_envs:
                raise ValueError(f"{name} must be a ({self.num_envs},) tensor on {self.device}")
            if t.dtype not in (torch.bool, torch.uint8):
                t = t.to(torch.uint8)
            return t.contiguous()

        flags = [flag(done, "done"), flag(is_goal, "is_goal"), flag(collision, "collision"),
                 flag(truncated, "truncated")]
        self._keep = flags  # alive until the kernel has read them
        out = _abi.OutT(None, *(t.data_ptr() for t in flags))
        with torch.cuda.device(self.device):
            _abi.check(self.lib.ffmp_episode_update(self.num_envs, C.byref(out), self.window, self.max_steps,
                                                    self.threshold, self._flags(), C.byref(self._ep_c),
                                                    self._stream()), "ffmp_episode_update")

    def update_from(self, env) -> None:
        """Update from an FFMPVec after its step() (reads its done / is_goal / collision / truncated)."""
        self.update(env.done, env.is_goal, env.collision, env.truncated)

    def summary(self) -> Dict[str, float]:
        """Running totals over all envs plus the mean reach rate (one small device->host copy)."""
        tot = self.totals.tolist()
        d = {k: int(v) for k, v in zip(TOTAL_KEYS, tot)}
        d["mean_reach_rate"] = float(self.reach_rate.mean().item()) if self.num_envs else 0.0
        d["any_complete"] = bool(self.complete.any().item()) if self.num_envs else False
        return d

    def state_dict(self) -> Dict[str, torch.Tensor]:
        keys = ("reach_bits", "reach_len", "reach_rate", "step", "episode", "total_step", "is_first", "complete",
                "totals")
        return {k: getattr(self, k).clone() for k in keys}

    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for k, v in sd.items():
            getattr(self, k).copy_(v)
