#!/usr/bin/env python3
"""A/B of the convolution kernels' launch variants — the MFMA shape (FFMP_TUNE_CONV_MFMA: 16 = 16x16x32,
32 = 32x32x16) and the kernel rows per ring step of the row-ring forward (FFMP_TUNE_CONV_KYS: 0 = by shape,
1, 2, 4) the B operand through LDS (FFMP_TUNE_CONV_LB), the weight gradient's operand prefetch (FFMP_TUNE_CONV_WGPF), B two taps ahead (FFMP_TUNE_CONV_BA2) the forward's position blocks per wave (FFMP_TUNE_CONV_MBW) its planar slots (FFMP_TUNE_CONV_PLANAR) pinned schedule (FFMP_TUNE_CONV_PIN) and the weight gradient's LDS-DMA stages (FFMP_TUNE_CONV_WGDMA) — on the reference Network's layers at batch B (default 256), random data, interleaved rounds in
ONE process (cdna_hip_programming.md rule 24): per layer and variant the median / min ms and PF/s over
the rounds, and each variant's max error against a float64 convolution of the same bf16 operands (first
4 samples).  Usage: python tools/conv_ab.py [B] [rounds] [variant ...]   (variant = mfma:kys:lb:wgpf:ba2:mbw:planar:pin:wgdma, e.g. 32:1:0:0:0:3:0:0:1)"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd import _abi  # noqa: E402
from flow_field_based_motion_planner_amd.conv_mfma import (conv2d_dgrad_nhwc, conv2d_nhwc, conv2d_wgrad_nhwc,  # noqa: E402
                                                          fold_input, frag_order, nhwc_bf16, pack_weight,
                                                          pack_weight_dgrad_bm, pack_weight_fold)

dev = torch.device("cuda:0")
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
ROUNDS = int(sys.argv[2]) if len(sys.argv) > 2 else 7
VARIANTS = [tuple(int(v) for v in (a + ":0:0:0:0:0:0:0:0").split(":")[:9]) for a in sys.argv[3:]] or \
    [(0, 0, 0, 0, 0, 0, 0, 0, 0), (0, 0, 0, 0, 0, 0, 0, 0, 1)]
torch.manual_seed(0)


def timeit(fn, reps=5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def rnd(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


layers = {}
# conv2: 32 -> 64, k 32, 69^2 -> 38^2 (forward, bias + ReLU, bf16 out)
x2 = torch.relu(rnd(B, 69, 69, 32))
w2 = rnd(64, 32, 32, 32, scale=1 / 181.0)
b2 = torch.randn(64, device=dev)
wp2 = pack_weight(w2)
layers["conv2 fwd"] = (2.0 * B * 38 * 38 * 64 * 32 * 32 * 32,
                       lambda: conv2d_nhwc(x2, wp2, b2, relu=True, out_dtype=torch.bfloat16),
                       lambda: F.relu(F.conv2d(x2[:4].permute(0, 3, 1, 2).double(), w2.double(), b2.double())))
# conv2's data gradient (samples as M) and weight gradient
g2 = rnd(B, 38, 38, 64)
wbm = pack_weight_dgrad_bm(w2)
layers["conv2 dgrad_bm"] = (2.0 * B * 38 * 38 * 64 * 32 * 32 * 32, lambda: conv2d_dgrad_nhwc(g2, wbm),
                            lambda: torch.ops.aten.convolution_backward(
                                g2[:4].permute(0, 3, 1, 2).double(), x2[:4].permute(0, 3, 1, 2).double(), w2.double(),
                                None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0])
layers["conv2 wgrad"] = (2.0 * B * 38 * 38 * 64 * 32 * 32 * 32, lambda: conv2d_wgrad_nhwc(g2, x2, 32, 32), None)
# conv3's weight gradient (64 -> 64, k 8, 38^2 -> 31^2)
g3 = rnd(B, 31, 31, 64)
x3w = torch.relu(rnd(B, 38, 38, 64))
layers["conv3 wgrad"] = (2.0 * B * 31 * 31 * 64 * 64 * 64, lambda: conv2d_wgrad_nhwc(g3, x3w, 8, 8), None)
# the folded conv1's weight gradient (32 folded channels, 32 x 2 taps at dx 16, 69^2 positions)
g1 = rnd(B, 69, 69, 32)
x1w = rnd(B, 100, 85, 32)
layers["conv1 wgrad (fold)"] = (2.0 * B * 69 * 69 * 32 * 32 * 32 * 2, lambda: conv2d_wgrad_nhwc(g1, x1w, 32, 2, dx=16), None)
# conv4's weight gradient (64 -> 64, k 8, 31^2 -> 24^2)
g4 = rnd(B, 24, 24, 64)
x4w = torch.relu(rnd(B, 31, 31, 64))
layers["conv4 wgrad"] = (2.0 * B * 24 * 24 * 64 * 64 * 64, lambda: conv2d_wgrad_nhwc(g4, x4w, 8, 8), None)
# conv1: 2 -> 32, k 32, 100^2 -> 69^2, folded (F = 16), bf16 out + ReLU
x1 = torch.rand(B, 2, 100, 100, device=dev) * 255
w1 = rnd(32, 2, 32, 32, scale=1 / 45.0)
b1 = torch.randn(32, device=dev)
wf1 = frag_order(pack_weight_fold(w1, 16))
layers["conv1 fwd (fold)"] = (2.0 * B * 69 * 69 * 32 * 2 * 32 * 32,
                              lambda: conv2d_nhwc(nhwc_bf16(x1), wf1, b1, relu=True, out_dtype=torch.bfloat16, dx=16,
                                                  x_fold=True), None)
# conv3's and conv4's data gradients (the small-image kernel with implicit padding k - 1)
from flow_field_based_motion_planner_amd.conv_mfma import pack_weight_dgrad  # noqa: E402
w3d = rnd(64, 64, 8, 8, scale=1 / 22.6)
wd3 = frag_order(pack_weight_dgrad(w3d))
gd3 = rnd(B, 31, 31, 64)
layers["conv3 dgrad (small)"] = (2.0 * B * 31 * 31 * 64 * 64 * 64, lambda: conv2d_nhwc(gd3, wd3, None, pad=7,
                                                                                       out_dtype=torch.bfloat16), None)
gd4 = rnd(B, 24, 24, 64)
layers["conv4 dgrad (small)"] = (2.0 * B * 24 * 24 * 64 * 64 * 64, lambda: conv2d_nhwc(gd4, wd3, None, pad=7,
                                                                                       out_dtype=torch.bfloat16), None)
# conv3: 64 -> 64, k 8, 38^2 -> 31^2 (small-image kernel, fragment-order weights)
x3 = torch.relu(rnd(B, 38, 38, 64))
w3 = rnd(64, 64, 8, 8, scale=1 / 22.6)
b3 = torch.randn(64, device=dev)
wf3 = frag_order(pack_weight(w3))
layers["conv3 fwd (small)"] = (2.0 * B * 31 * 31 * 64 * 64 * 64, lambda: conv2d_nhwc(x3, wf3, b3, relu=True,
                                                                                     out_dtype=torch.bfloat16),
                               lambda: F.relu(F.conv2d(x3[:4].permute(0, 3, 1, 2).double(), w3.double(), b3.double())))

lib = _abi.load()
def setv(v):
    lib.ffmp_set_tuning(_abi.TUNE_CONV_MFMA, v[0])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_KYS, v[1])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_LB, v[2])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_WGPF, v[3])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_BA2, v[4])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_MBW, v[5])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_PLANAR, v[6])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_PIN, v[7])
    lib.ffmp_set_tuning(_abi.TUNE_CONV_WGDMA, v[8])


res = {k: {s: [] for s in VARIANTS} for k in layers}
errs = {k: {} for k in layers}
for s in VARIANTS:  # correctness per variant (and warm-up)
    setv(s)
    for k, (flop, fn, ref) in layers.items():
        out = fn()
        torch.cuda.synchronize()
        if ref is not None:
            r = ref()
            o = out[:4].double()
            if o.shape != r.shape:
                o = o.permute(0, 3, 1, 2)
            errs[k][s] = float((o - r).abs().max() / (r.abs().max() + 1e-9))
for rnd_i in range(ROUNDS):
    for s in VARIANTS:
        setv(s)
        for k, (flop, fn, ref) in layers.items():
            res[k][s].append(timeit(fn))
setv((0, 0, 0, 0, 0, 0, 0, 0, 0))
for k, (flop, fn, ref) in layers.items():
    line = [f"{k:20s} B={B}"]
    for s in VARIANTS:
        v = sorted(res[k][s])
        med = v[len(v) // 2]
        line.append(f"{':'.join(map(str, s))}: med {med:.4f} ms min {v[0]:.4f} ({flop / med / 1e12:.3f} PF/s) err {errs[k].get(s, float('nan')):.2e}")
    print(" | ".join(line), flush=True)
