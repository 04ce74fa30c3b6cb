"""Brain — the reference's double-DQN learner (src/train.py:306-431), batched over FFMPVec envs.

Everything stays in HBM: transitions go into the device ReplayMemory (records), minibatches
are re-rastered there, and the Q-networks run on the batch without host round trips.

  Brain.__init__ (:307-314)                     -> same hyper-parameters (train.py:59-79)
  Brain.decide_action (:336-347)                -> decide_action(obs, episode): per-env
      epsilon = 0.5 * (1 / (episode + 1)); greedy iff epsilon <= U(0,1); batched, per_sample
      coupling (= the reference's B = 1 forward for every env)
  Brain.replay (:316-333) + make_minibatch (:349-369)
      + get_expected_state_action_values (:371-411) + update_main_q_network (:413-428)
                                                -> replay(): sample, Q(s,a), a* = argmax_a
      Q_main(s',a), y = r + GAMMA * Q_target(s', a*) (no terminal mask, as the reference;
      mask_terminal=True multiplies by 1 - done), MSE, Adam step
  Brain.update_target_q_network (:430-431)      -> same

input_channels (train.py:66-69): 2 (default, the configuration train.py runs) = [older, newest];
1 = the newest frame; 3 = the newest frame + the env's flow planes (network.map_channels), as the
option comments describe them.  temporal_maps=True instead takes make_temporal_maps' code path for
a mono BEV image (train.py:474-486: map_memory holds INPUT_CHANNELS frames): input_channels = k
frames, oldest first, served from the env's frame ring (FFMPVec.temporal_maps, k <= frame_window)
and re-rastered by the replay memory (ReplayMemory(series=k)).  input_channels=12 is the option
comment's "(occupancy(MONO) + flow(RGB)) * series(3 steps)" (train.py:66): three 4-channel BEV
images [occupancy, R, G, B] from an env built with FFMPVec(bev_series=3) (FFMPVec.bev_maps; the RGB
encoding is include/ffmp.h ffmp_bev_image's), replayed by ReplayMemory(series=3, bev=True).

amp=True (not the reference's arithmetic, opt-in): the Q-network forwards (acting, replay and
target) run under torch.autocast bfloat16 — the convolutions on the MFMA units in bf16, fp32
accumulation, fp32 master weights, Adam state and loss (tests/test_gpu_learner.py bounds the
difference to the fp32 update).  With amp, conv2-conv4 (and conv2's data gradient, ~80 % of the
network's FLOPs) run on the hand-written MFMA kernel (conv_mfma.py; mfma=False: MIOpen's).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn as nn

from .conv_mfma import track_optimizer
from .network import Network, map_channels
from .replay import ReplayMemory

GAMMA = 0.95            # train.py:59
BATCH_SIZE = 1024       # train.py:63
CAPACITY = 20000        # train.py:65
LEARNING_RATE = 0.0005  # train.py:71
NUM_ACTIONS = 28        # train.py:70
INPUT_CHANNELS = 2      # train.py:69


class Brain:
    def __init__(self, env, capacity: int = CAPACITY, batch_size: int = BATCH_SIZE, gamma: float = GAMMA,
                 lr: float = LEARNING_RATE, replay_coupling: str = "reference", mask_terminal: bool = False,
                 seed: int = 0, amp: bool = False, channels_last: bool = False,
                 input_channels: int = INPUT_CHANNELS, mfma: Optional[bool] = None, temporal_maps: bool = False):
        self.env = env
        self.device = env.device
        self.num_actions = NUM_ACTIONS
        self.batch_size, self.gamma, self.mask_terminal = int(batch_size), float(gamma), bool(mask_terminal)
        self.replay_coupling = replay_coupling
        self.amp = bool(amp)
        self.mfma = self.amp if mfma is None else bool(mfma)  # effective under amp only (network.py)
        self.channels_last = bool(channels_last)
        # map input per train.py:66-69 (network.map_channels): 2 = [older, newest] (default), 1 =
        # newest frame, 3 = newest frame + flow xy (needs the env's flow planes)
        self.input_channels = int(input_channels)
        self.temporal_maps = bool(temporal_maps)
        self.bev = self.input_channels == 12
        if self.bev:
            if self.temporal_maps:
                raise ValueError("input_channels=12 is the BEV series (occupancy + RGB flow x 3 steps); "
                                 "temporal_maps is the mono-frame series")
            if getattr(env, "bev", None) is None or env.bev_series < 3:
                raise ValueError("input_channels=12 needs FFMPVec(..., FFMPConfig(flow=True), bev_series=3)")
        elif self.temporal_maps:
            if not 1 <= self.input_channels <= env.max_temporal_frames:
                raise ValueError(f"temporal_maps: input_channels must be in [1, {env.max_temporal_frames}] for this "
                                 f"env (frame_window={env.frame_window}, ring={env.ring}; a wrapping ring holds "
                                 f"W - 1 distinct frames)")
        else:
            if self.input_channels == 3 and not env.cfg.flow:
                raise ValueError("input_channels=3 needs an env with FFMPConfig(flow=True)")
            if self.input_channels not in (1, 2, 3):
                raise ValueError("input_channels must be 1, 2 or 3")
        series = 3 if self.bev else self.input_channels if self.temporal_maps else 2
        self.memory = ReplayMemory(env, max(int(capacity), env.num_envs), seed=seed, series=series, bev=self.bev)
        g = env.cfg.grid
        with torch.random.fork_rng(devices=[]):  # seeded init without touching the caller's RNG
            torch.manual_seed(seed)
            self.main_q_network = Network(self.input_channels, NUM_ACTIONS, grid=g, mfma=self.mfma).to(self.device)
            self.target_q_network = Network(self.input_channels, NUM_ACTIONS, grid=g, mfma=self.mfma).to(self.device)
        if self.channels_last:  # NHWC convolutions (same values; MIOpen picks other kernels)
            self.main_q_network.to(memory_format=torch.channels_last)
            self.target_q_network.to(memory_format=torch.channels_last)
        # torch's fused Adam on the GPU: one kernel per step instead of the foreach chain (~7 launches,
        # ~0.15 ms per update at the reference's Network), the same update up to fp32 rounding
        self.optimizer = torch.optim.Adam(self.main_q_network.parameters(), lr=lr,
                                          fused=self.device.type == "cuda")
        # the fused step writes the weights without bumping their version counters: bump them after
        # every step, or the MFMA convolutions' cached bf16 weight packs would go stale
        track_optimizer(self.optimizer)
        self.loss: Optional[torch.Tensor] = None
        self.step = 0
        self.gen = torch.Generator(device=self.device)
        self.gen.manual_seed(int(seed) + 1)

    def _q(self, net: Network, coupling: str, sm, sg, sv, st, flow=None):
        if self.temporal_maps or self.bev:  # already the k frames / the 12 BEV channels
            sm = sm.float() if sm.dtype == torch.uint8 else sm
        else:
            sm = map_channels(sm, flow, self.input_channels)  # uint8 frames (u8f16 layout) -> float 0 / 255
        if self.channels_last:
            sm = sm.contiguous(memory_format=torch.channels_last)
        prev, net.coupling = net.coupling, coupling
        try:
            with torch.autocast(device_type="cuda", dtype=torch.bfloat16, enabled=self.amp):
                return net(sm, sg, sv, st).float()
        finally:
            net.coupling = prev

    def decide_action(self, obs: Dict[str, torch.Tensor], episode: torch.Tensor) -> torch.Tensor:
        """Epsilon-greedy actions (N,) int64 for every env (train.py:336-347).  With temporal_maps
        the map input is the env's k-frame series (FFMPVec.temporal_maps), not obs["state_m"]."""
        n = obs["state_m"].shape[0]
        if self.temporal_maps:
            obs = dict(obs, state_m=self.env.temporal_maps(self.input_channels))
        elif self.bev:
            obs = dict(obs, state_m=self.env.bev_maps(3))
        epsilon = 0.5 * (1.0 / (episode.to(torch.float64) + 1.0))
        u = torch.rand(n, generator=self.gen, device=self.device, dtype=torch.float64)
        self.main_q_network.eval()
        with torch.no_grad():
            q = self._q(self.main_q_network, "per_sample", obs["state_m"], obs["state_g"], obs["state_v"],
                        obs["state_t"], obs.get("flow"))
        greedy = q.max(1)[1]
        rand = torch.randint(0, self.num_actions, (n,), generator=self.gen, device=self.device)
        return torch.where(epsilon <= u, greedy, rand)

    def replay(self, index: Optional[torch.Tensor] = None) -> Optional[torch.Tensor]:
        """One learner update; None until the memory holds a minibatch (train.py:319-320)."""
        if len(self.memory) < self.batch_size and index is None:
            return None
        b, ex = self.memory.sample(self.batch_size, index=index)
        c = self.replay_coupling
        self.main_q_network.eval()
        self.target_q_network.eval()
        fs, fo = ex.get("flow"), ex.get("observe_flow")
        sav = self._q(self.main_q_network, c, b.state_m, b.state_g, b.state_v, b.state_t, fs).gather(1, b.action)
        with torch.no_grad():
            a_m = self._q(self.main_q_network, c, b.observe_m, b.observe_g, b.observe_v, b.observe_t, fo).max(1)[1]
            nxt = self._q(self.target_q_network, c, b.observe_m, b.observe_g, b.observe_v,
                          b.observe_t, fo).gather(1, a_m.view(-1, 1)).squeeze(1)
            if self.mask_terminal:
                nxt = nxt * (~ex["done"]).to(nxt.dtype)
            expected = b.reward + self.gamma * nxt
        self.main_q_network.train()
        loss = nn.functional.mse_loss(sav, expected.unsqueeze(1))
        self.loss = loss
        self.optimizer.zero_grad()
        loss.backward()
        self.optimizer.step()
        return loss.detach()

    def update_target_q_network(self) -> None:
        self.target_q_network.load_state_dict(self.main_q_network.state_dict())
