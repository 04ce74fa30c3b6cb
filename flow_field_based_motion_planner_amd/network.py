"""Network — the reference's dueling Q-network (src/train.py:231-303), batched on the GPU.

Same layers, names and shapes as the reference, so its state_dict (and checkpoints, loaded
with `torch.load(..., weights_only=True)`) load unchanged.  What changes is how the forward
runs on a batch of env tensors already in HBM:

  * no host round trips: the reference moves x_m / the tile / adv / val to the CPU and back
    (:271-274, :296-300); here everything stays on the device;
  * the fc1 "tile" (:261-267) is one gather: the loop `for i in range(grid_num): value =
    x_gvt_[0][i]; tile = full((convw, convh), value)` keeps only its LAST value, i.e. feature
    convw-1 of batch element 0, added to every cell of every channel of every sample.
    `coupling="reference"` (default) reproduces that exactly, including the cross-sample
    coupling at B > 1; `coupling="per_sample"` uses each sample's own feature, which is what
    the reference computes for B = 1 (its acting path) and keeps samples independent.

The linears are library GEMMs (hipBLASLt through torch).  With `mfma=True` and under bfloat16
autocast (Brain(amp=True)), every convolution + ReLU runs on the hand-written MFMA kernels instead
of MIOpen (conv_mfma.py, include/ffmp.h ffmp_conv2d_fwd_bf16 / ffmp_conv2d_dgrad_bf16 /
ffmp_conv2d_wgrad_bf16: the forward, the data gradient and the weight gradient; conv1's 1-16 map
channels — the reference's 1 / 2 / 3 and the 12-channel BEV series, conv_mfma.fold_supported — with
its kernel columns folded into 32 channels, its input gradient — never needed by the Network — MIOpen's):
bf16 operands and fp32 accumulation like autocast's conv2d (the bias added in fp32, where
autocast rounds it to bf16 first).  A layer whose input shape the kernels do not take
(conv_mfma.supported / fold_supported with the shape: e.g. 64-channel rows over 16 KiB at
G >= 191, weight-gradient rows under 8 positions at G 91-97, a batch over 65,535) runs
F.relu(conv(x)) under autocast instead.
Input maps must be G x G with G - 90 > 0 (conv k=32,32,8 then conv4 k=8 three times); the
reference's fc2 (6400 inputs) fixes G = 100, other G size fc2 accordingly.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import conv_mfma


class Network(nn.Module):
    def __init__(self, input_channels: int = 2, outputs: int = 28, grid: int = 100, coupling: str = "reference",
                 mfma: bool = False):
        super().__init__()
        self.mfma = bool(mfma)
        if coupling not in ("reference", "per_sample"):
            raise ValueError("coupling must be 'reference' or 'per_sample'")
        side = grid - 31 - 31 - 7 - 3 * 7
        if side <= 0:
            raise ValueError(f"grid {grid} too small for the reference's convolution stack (needs > 90)")
        conv3_side = grid - 31 - 31 - 7
        if conv3_side > 67:
            raise ValueError(f"grid {grid}: the fc1 tile reads feature {conv3_side - 1} of 67 (needs grid <= 136)")
        self.coupling = coupling
        self.grid = grid
        self.conv1 = nn.Conv2d(input_channels, 32, kernel_size=32)
        self.conv2 = nn.Conv2d(32, 64, kernel_size=32)
        self.conv3 = nn.Conv2d(64, 64, kernel_size=8)
        self.conv4 = nn.Conv2d(64, 64, kernel_size=8)
        self.fc1 = nn.Linear(5, 67)
        self.fc2 = nn.Linear(64 * side * side, 512)
        self.fc3 = nn.Linear(512, 512)
        self.fc4_ea = nn.Linear(512, outputs)  # A(s, a)
        self.fc4_ev = nn.Linear(512, 1)        # V(s)

    def _conv_relu(self, conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
        """relu(conv(x)): on the MFMA kernel when enabled, under bf16 autocast, for its shapes."""
        if self.mfma and x.is_cuda and torch.is_autocast_enabled("cuda") and \
                torch.get_autocast_dtype("cuda") == torch.bfloat16:
            if conv_mfma.supported(conv, x.shape):
                return conv_mfma.conv_relu(conv, x)
            if conv_mfma.fold_supported(conv, x.shape):  # conv1: 1-16 map channels (padded to 2^k)
                return conv_mfma.fold_conv_relu(conv, x)
        return F.relu(conv(x))

    def forward(self, state_m: torch.Tensor, state_g: torch.Tensor, state_v: torch.Tensor,
                state_t: torch.Tensor) -> torch.Tensor:
        x_m = self._conv_relu(self.conv1, state_m)
        x_m = self._conv_relu(self.conv2, x_m)
        x_m = self._conv_relu(self.conv3, x_m)
        x_gvt = F.relu(self.fc1(torch.cat((state_g, state_v, state_t), 1)))
        tile = x_gvt[:, x_m.shape[2] - 1]                      # the loop's last value (:263-267)
        if self.coupling == "reference":
            tile = tile[:1].expand(x_m.shape[0])               # x_gvt_[0][...]: batch element 0
        x = x_m + tile.view(-1, 1, 1, 1)
        x = self._conv_relu(self.conv4, x)
        x = self._conv_relu(self.conv4, x)
        x = self._conv_relu(self.conv4, x)
        x = torch.flatten(x, start_dim=1)
        x = F.relu(self.fc2(x))
        x = F.relu(self.fc3(x))
        adv = self.fc4_ea(x)
        val = self.fc4_ev(x)
        return adv + val - adv.mean(1, keepdim=True).expand(-1, adv.size(1))


def map_channels(state_m: torch.Tensor, flow: "torch.Tensor | None", channels: int = 2) -> torch.Tensor:
    """The map input of the reference's INPUT_CHANNELS options (src/train.py:66-69):
      2  two steps of temporal_bev_image, [older, newest] — the configuration train.py runs (:69)
      1  only temporal_bev_image: the newest frame (:68)
      3  (occupancy(MONO) + flow(xy)) * series(1 steps) (:67): the newest frame, then the BEV
         motion-flow planes (FFMPVec with cfg.flow: per-cell ego velocity of the covering disc)
    (:66's 12 channels, occupancy + RGB flow over 3 steps, are a series, not a view of one
    observation: FFMPVec(bev_series=3).bev_maps() / Brain(input_channels=12).)  uint8 frames (the
    compact layout) come back as float with the same 0 / 255 values."""
    if state_m.dtype == torch.uint8:
        state_m = state_m.float()
    if channels == 2:
        return state_m
    if channels == 1:
        return state_m[:, 1:2]
    if channels == 3:
        if flow is None:
            raise ValueError("3 map channels need the flow planes (FFMPConfig(flow=True))")
        return torch.cat((state_m[:, 1:2], flow.float()), 1)  # binary16 flow (u8f16 layout) -> float
    raise ValueError(f"map channels must be 1, 2 or 3 (train.py:67-69; the 12-channel option is "
                     f"FFMPVec.bev_maps), got {channels}")

