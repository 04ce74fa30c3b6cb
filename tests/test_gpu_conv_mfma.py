"""The learner's MFMA convolution (include/ffmp.h ffmp_conv2d_fwd_bf16, conv_mfma.py) against a
float64 convolution of the same bf16 operands (torch's native GPU path, MIOpen off), and the
autograd function against autocast's bf16 conv2d.  Shapes: the reference Network's conv2
(/root/reference/src/train.py:235: 32 -> 64 channels, k = 32, 69^2 -> 38^2), conv3/conv4-like
(64 -> 64, k = 8), the transposed conv2 a data gradient runs (64 -> 32 over a 100^2 padded image),
and ragged sizes whose position count is not a multiple of the 512-position tile.

Tolerance (fp32 accumulation of up to 32,768 bf16 products, exact in fp32): |y - y64| <=
5e-5 * (|x| * |w|)(same position) + 1e-6; a layout error is O(1) relative."""
import pytest
import torch
import torch.nn.functional as F

from flow_field_based_motion_planner_amd.conv_mfma import MFMAConv2dReLU, conv2d_nhwc, frag_order, pack_weight

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _ref64(xb, wp, bias, pad=0):
    x = xb.double().permute(0, 3, 1, 2)
    w = wp.double().permute(2, 3, 0, 1)
    with torch.backends.cudnn.flags(enabled=False):
        y = F.conv2d(x, w, None if bias is None else bias.double(), padding=pad)
        a = F.conv2d(x.abs(), w.abs(), padding=pad)
    return y.permute(0, 2, 3, 1), a.permute(0, 2, 3, 1)


@pytest.mark.parametrize("B,H,W,C,K,N,pad", [
    (2, 69, 69, 32, 32, 64, 0),   # conv2
    (3, 38, 38, 64, 8, 64, 0),    # conv3 / conv4
    (1, 100, 100, 64, 32, 32, 0),
    (2, 38, 38, 64, 32, 32, 31),  # conv2's data gradient (implicit padding k - 1)
    (2, 40, 45, 32, 5, 32, 0), (1, 31, 31, 64, 8, 64, 0), (5, 33, 70, 32, 2, 64, 0), (3, 20, 24, 32, 5, 64, 2),
    # the row-ring kernel with padding at each tile size (512 / 256 / 128 positions)
    (2, 30, 30, 64, 3, 64, 2), (2, 12, 12, 64, 2, 64, 1), (2, 10, 10, 32, 2, 32, 1),
    # the small-image kernel on data-gradient shapes: conv3's and conv4's (k - 1 = 7 zero cells)
    (2, 31, 31, 64, 8, 64, 7), (2, 10, 10, 64, 8, 64, 7),
    # the 4 x 8 patch kernel of the data gradient (round 4) on ragged outputs: heights not a multiple
    # of 4, widths not a multiple of 8, patches past the image, each patches-per-workgroup choice
    (1, 50, 45, 64, 6, 32, 5), (2, 45, 9, 32, 3, 64, 2), (1, 47, 33, 32, 7, 32, 6), (3, 60, 61, 64, 17, 64, 16)])
def test_conv_fwd_matches_float64(B, H, W, C, K, N, pad):
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + H + K)
    xb = torch.randn((B, H, W, C), device=DEV, generator=g).to(torch.bfloat16)
    w = torch.randn((N, C, K, K), device=DEV, generator=g) / (C * K * K) ** 0.5
    bias = torch.randn(N, device=DEV, generator=g) * 0.1
    wp = pack_weight(w)
    y = conv2d_nhwc(xb, wp, bias, pad=pad)
    ref, absref = _ref64(xb, wp, bias, pad)
    assert y.shape == (B, H + 2 * pad - K + 1, W + 2 * pad - K + 1, N)
    err = (y.double() - ref).abs()
    bad = err > 5e-5 * absref + 1e-6
    assert not bool(bad.any()), f"{int(bad.sum())} of {bad.numel()} outside tolerance, max err {float(err.max())}"
    # fused ReLU + bf16 output: the same fp32 accumulator, rounded
    yb = conv2d_nhwc(xb, wp, bias, relu=True, out_dtype=torch.bfloat16, pad=pad)
    assert torch.equal(yb, torch.relu(y).to(torch.bfloat16))
    # the weight in fragment order (FFMP_CONV_W_FRAG): the same products in the same order, bit for bit
    wf = frag_order(wp)
    assert torch.equal(conv2d_nhwc(xb, wf, bias, pad=pad), y)
    assert torch.equal(conv2d_nhwc(xb, wf, bias, relu=True, out_dtype=torch.bfloat16, pad=pad), yb)


@pytest.mark.parametrize("B,C,H,N,K", [(4, 32, 69, 64, 32),   # conv2
                                       (3, 64, 38, 64, 8),    # conv3
                                       (3, 64, 31, 64, 8), (2, 64, 24, 64, 8), (3, 64, 17, 64, 8)])  # conv4 x 3
def test_autograd_function_against_autocast_and_float64(B, C, H, N, K):
    """relu(conv) of the reference Network's conv2 / conv3 / conv4 shapes: the forward within bf16
    rounding of autocast's conv2d; the gradients (input: the MFMA data-gradient kernel — samples as M
    where ffmp_conv2d_dgrad_bf16 takes the shape, else the padded full convolution; weight: the MFMA
    weight-gradient kernel; bias: an fp32 sum; all masked by the kernel's own output) against float64
    autograd of the same masked product."""
    g = torch.Generator(device=DEV).manual_seed(7 + H)
    conv = torch.nn.Conv2d(C, N, kernel_size=K).to(DEV)
    x = torch.relu(torch.randn((B, C, H, H), device=DEV, generator=g)).to(torch.bfloat16).requires_grad_(True)
    y = MFMAConv2dReLU.apply(x, conv.weight, conv.bias)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y2 = F.relu(conv(x))
    assert y.shape == y2.shape and y.dtype == y2.dtype == torch.bfloat16
    diff = (y.detach().float() - y2.float()).abs()
    assert float(diff.max()) <= 0.02 * float(y2.float().abs().max())
    gy = torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16)
    y.backward(gy)
    gw, gb, gx = conv.weight.grad, conv.bias.grad, x.grad
    assert gw.dtype == torch.float32 and gb.dtype == torch.float32 and gx.dtype == torch.bfloat16
    # float64 reference: d/d(x, w, b) of sum(conv(x, w_bf16, b) * gy * [y > 0])
    x64 = x.detach().double().requires_grad_(True)
    w64 = conv.weight.detach().to(torch.bfloat16).double().requires_grad_(True)
    b64 = conv.bias.detach().double().requires_grad_(True)
    with torch.backends.cudnn.flags(enabled=False):
        z = F.conv2d(x64, w64, b64)
    (z * gy.double() * (y.detach() > 0)).sum().backward()
    for got, ref in ((gw, w64.grad), (gb, b64.grad), (gx, x64.grad)):
        err = (got.double() - ref).abs()
        assert float(err.max()) <= 0.01 * float(ref.abs().max()) + 1e-6, (float(err.max()), float(ref.abs().max()))


def test_network_mfma_against_miopen_under_autocast():
    """The reference Network (B = 6, 100^2 maps) with conv2-conv4 on the MFMA kernel against the
    same weights through MIOpen, both under bf16 autocast: Q-values within bf16 tolerance, and every
    parameter gradient of a loss on them in the same direction (cosine >= 0.99) and of the same norm
    (within 5 %).  (Elementwise agreement is not expected deep in the backward pass: the two paths
    round each activation to bf16 independently, so ReLU masks differ where a value is ~0.)"""
    from flow_field_based_motion_planner_amd.network import Network
    g = torch.Generator(device=DEV).manual_seed(11)
    torch.manual_seed(11)
    a = Network(2, 28, mfma=True).to(DEV)
    b = Network(2, 28, mfma=False).to(DEV)
    b.load_state_dict(a.state_dict())
    sm = (torch.rand((6, 2, 100, 100), device=DEV, generator=g) > 0.9).float() * 255
    sg, sv, st = (torch.rand((6, k), device=DEV, generator=g) for k in (2, 2, 1))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        qa = a(sm, sg, sv, st).float()
        qb = b(sm, sg, sv, st).float()
    assert float((qa - qb).abs().max()) <= 0.03 * float(qb.abs().max()) + 1e-3
    (qa ** 2).mean().backward()
    (qb ** 2).mean().backward()
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        ga, gb = pa.grad.double().flatten(), pb.grad.double().flatten()
        cos = float(ga @ gb / (ga.norm() * gb.norm() + 1e-30))
        rel = float((ga.norm() - gb.norm()).abs() / (gb.norm() + 1e-30))
        assert cos >= 0.99 and rel <= 0.05, (name, cos, rel)


@pytest.mark.parametrize("B,H,W,KH,KW,dx,N", [(2, 40, 85, 32, 2, 16, 32), (3, 30, 70, 7, 3, 8, 64)])
def test_conv_dilated_matches_float64(B, H, W, KH, KW, dx, N):
    """Kernel columns dx cells apart (the folded form of a few-channel convolution)."""
    g = torch.Generator(device=DEV).manual_seed(H + W)
    xb = torch.randn((B, H, W, 32), device=DEV, generator=g).to(torch.bfloat16)
    w = torch.randn((N, 32, KH, KW), device=DEV, generator=g) / (32 * KH * KW) ** 0.5
    y = conv2d_nhwc(xb, pack_weight(w), None, dx=dx)
    x64 = xb.double().permute(0, 3, 1, 2)
    w64 = w.to(torch.bfloat16).double()
    with torch.backends.cudnn.flags(enabled=False):
        ref = F.conv2d(x64, w64, dilation=(1, dx)).permute(0, 2, 3, 1)
        absref = F.conv2d(x64.abs(), w64.abs(), dilation=(1, dx)).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    assert not bool(((y.double() - ref).abs() > 5e-5 * absref + 1e-6).any())
    assert torch.equal(conv2d_nhwc(xb, frag_order(pack_weight(w)), None, dx=dx), y)  # FFMP_CONV_W_FRAG


@pytest.mark.parametrize("C", [2, 1, 3, 12])
def test_folded_conv1_against_float64(C):
    """The reference Network's conv1 (C map channels -> 32, k = 32, 100^2 -> 69^2; train.py:234)
    with its kernel columns folded into 32 channels: forward vs float64 of the same bf16 operands
    (then ReLU, bf16), weight / bias gradients vs float64 autograd of the masked product."""
    from flow_field_based_motion_planner_amd.conv_mfma import fold_conv_relu, fold_supported
    g = torch.Generator(device=DEV).manual_seed(5 + C)
    conv = torch.nn.Conv2d(C, 32, kernel_size=32).to(DEV)
    assert fold_supported(conv)
    x = (torch.rand((3, C, 100, 100), device=DEV, generator=g) > 0.85).float() * 255
    y = fold_conv_relu(conv, x)  # C = 3: a zero fourth channel; C = 12: four zero channels (F = 2)
    x64 = x.double()
    w64 = conv.weight.detach().to(torch.bfloat16).double().requires_grad_(True)
    b64 = conv.bias.detach().double().requires_grad_(True)
    with torch.backends.cudnn.flags(enabled=False):
        z = F.conv2d(x64, w64, b64)
        absz = F.conv2d(x64, w64.detach().abs()) + b64.detach().abs().view(1, -1, 1, 1)
    want = torch.relu(z.detach())
    assert y.shape == want.shape and y.dtype == torch.bfloat16
    tol = 5e-5 * absz + 1e-6 + want.abs() * 2 ** -8  # + the bf16 rounding of the output
    assert not bool(((y.double() - want).abs() > tol).any())
    gy = torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16)
    y.backward(gy)
    (z * gy.double() * (y.detach() > 0)).sum().backward()
    for got, ref in ((conv.weight.grad, w64.grad), (conv.bias.grad, b64.grad)):
        err = (got.double() - ref).abs()
        assert float(err.max()) <= 0.01 * float(ref.abs().max()) + 1e-6


@pytest.mark.parametrize("B,H,W,C,KH,KW,N,dx", [
    (3, 69, 69, 32, 32, 32, 64, 1),   # conv2
    (3, 38, 38, 64, 8, 8, 64, 1),     # conv3
    (2, 17, 17, 64, 8, 8, 64, 1),     # conv4's last
    (2, 100, 85, 32, 32, 2, 32, 16),  # conv1 folded (2 channels, 16 kernel columns per folded column)
    (2, 20, 20, 64, 8, 8, 32, 1), (3, 20, 22, 32, 6, 4, 32, 1)])
def test_wgrad_matches_float64(B, H, W, C, KH, KW, N, dx):
    """ffmp_conv2d_wgrad_bf16 (positions along k through ds_read_b64_tr_b16) against torch's float64
    weight gradient of the same bf16 operands; tolerance as the forward's."""
    from flow_field_based_motion_planner_amd.conv_mfma import conv2d_wgrad_nhwc
    g0 = torch.Generator(device=DEV).manual_seed(B + H + KH + N)
    Ho, Wo = H - KH + 1, W - (KW - 1) * dx
    x = torch.randn((B, H, W, C), device=DEV, generator=g0).to(torch.bfloat16)
    g = torch.randn((B, Ho, Wo, N), device=DEV, generator=g0).to(torch.bfloat16)
    dw = conv2d_wgrad_nhwc(g, x, KH, KW, dx=dx)
    assert dw.shape == (KH, KW, N, C) and dw.dtype == torch.float32
    x64, g64 = x.double().permute(0, 3, 1, 2), g.double().permute(0, 3, 1, 2)
    with torch.backends.cudnn.flags(enabled=False):
        ref = torch.nn.grad.conv2d_weight(x64, (N, C, KH, KW), g64, dilation=(1, dx)).permute(2, 3, 0, 1)
        absref = torch.nn.grad.conv2d_weight(x64.abs(), (N, C, KH, KW), g64.abs(), dilation=(1, dx)).permute(2, 3, 0, 1)
    err = (dw.double() - ref).abs()
    bad = err > 5e-5 * absref + 1e-6
    assert not bool(bad.any()), f"{int(bad.sum())} of {bad.numel()} outside tolerance, max err {float(err.max())}"


@pytest.mark.parametrize("B,Hy,Wy,C,KH,KW,N", [
    (2, 38, 38, 64, 32, 32, 32),    # conv2's data gradient (the reference Network, train.py:235)
    (33, 38, 38, 64, 32, 32, 32),   # a ragged second sample group (one sample)
    (64, 38, 38, 64, 32, 32, 32),   # two full groups
    (3, 38, 38, 32, 32, 32, 32),    # 32 gradient channels: one phase per kernel row
    (5, 20, 24, 64, 5, 7, 32),      # a small kernel: pieces left after the kernel-column sweep
    (2, 7, 40, 64, 3, 33, 32),      # the widest gradient rows (LDS) and output rows of 72 positions
    (4, 1, 1, 32, 2, 3, 32)])       # a single gradient cell
def test_dgrad_samples_as_m_matches_float64(B, Hy, Wy, C, KH, KW, N):
    """ffmp_conv2d_dgrad_bf16 (32 samples per MFMA block, every tap of every position exact) against
    torch's float64 input gradient of the same bf16 operands (torch.nn.grad.conv2d_input); the
    forward's tolerance.  The bf16 output is the fp32 result rounded."""
    from flow_field_based_motion_planner_amd.conv_mfma import conv2d_dgrad_nhwc, dgrad_bm_ok, pack_weight_dgrad_bm
    assert dgrad_bm_ok(B, Hy, Wy, C, KH, KW, N)
    g0 = torch.Generator(device=DEV).manual_seed(B + Hy + KW + C)
    g = torch.randn((B, Hy, Wy, C), device=DEV, generator=g0).to(torch.bfloat16)
    w = torch.randn((C, N, KH, KW), device=DEV, generator=g0) / (C * KH * KW) ** 0.5  # forward: N -> C channels
    wb = pack_weight_dgrad_bm(w)
    dx = conv2d_dgrad_nhwc(g, wb, out_dtype=torch.float32)
    Hx, Wx = Hy + KH - 1, Wy + KW - 1
    assert dx.shape == (B, Hx, Wx, N)
    g64, w64 = g.double().permute(0, 3, 1, 2), w.to(torch.bfloat16).double()
    with torch.backends.cudnn.flags(enabled=False):
        ref = torch.nn.grad.conv2d_input((B, N, Hx, Wx), w64, g64).permute(0, 2, 3, 1)
        absref = torch.nn.grad.conv2d_input((B, N, Hx, Wx), w64.abs(), g64.abs()).permute(0, 2, 3, 1)
    err = (dx.double() - ref).abs()
    bad = err > 5e-5 * absref + 1e-6
    assert not bool(bad.any()), f"{int(bad.sum())} of {bad.numel()} outside tolerance, max err {float(err.max())}"
    assert torch.equal(conv2d_dgrad_nhwc(g, wb), dx.to(torch.bfloat16))


def test_dgrad_samples_as_m_shape_limits():
    """The launch's own checks (ffmp_conv2d_check kind 2): 32-channel outputs only, output rows of at
    most 72 positions, two gradient rows within the LDS."""
    from flow_field_based_motion_planner_amd.conv_mfma import dgrad_bm_ok
    assert dgrad_bm_ok(256, 38, 38, 64, 32, 32, 32) and dgrad_bm_ok(1024, 38, 38, 64, 32, 32, 32)
    assert not dgrad_bm_ok(256, 31, 31, 64, 8, 8, 64)   # conv3's: 64 output channels
    assert not dgrad_bm_ok(2, 5, 10, 64, 3, 64, 32)     # output rows of 73 positions
    assert not dgrad_bm_ok(2, 10, 41, 64, 3, 3, 32)     # 41 columns x 2 KiB x 2 rows > 160 KiB


@pytest.mark.parametrize("Cc", [2, 4, 16])
@pytest.mark.parametrize("wide", [False, True])  # the small-image kernel / the row-ring kernel
def test_conv_x_fold_equals_materialized_fold(Cc, wide):
    """FFMP_CONV_X_FOLD: the kernel folding the unfolded NHWC input on the fly == the same launch on
    fold_input's materialized copy, bit for bit (plain and fragment-order weights)."""
    from flow_field_based_motion_planner_amd.conv_mfma import fold_input, pack_weight_fold, small_route
    F = 32 // Cc
    g = torch.Generator(device=DEV).manual_seed(Cc)
    x = torch.randn((3, Cc, 45, 100 if wide else 37 + F), device=DEV, generator=g)
    assert small_route(45, x.shape[3] - F + 1, 32, 5, 2, 0, F) != wide
    w = torch.randn((32, Cc, 5, 2 * F), device=DEV, generator=g) / (Cc * 10 * F) ** 0.5
    bias = torch.randn(32, device=DEV, generator=g)
    wp = pack_weight_fold(w, F)
    xn = x.to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    for wk in (wp, frag_order(wp)):
        ref = conv2d_nhwc(fold_input(x, F), wk, bias, relu=True, out_dtype=torch.bfloat16, dx=F)
        got = conv2d_nhwc(xn, wk, bias, relu=True, out_dtype=torch.bfloat16, dx=F, x_fold=True)
        assert got.shape == ref.shape and torch.equal(got, ref)


@pytest.fixture
def conv_knobs():
    from flow_field_based_motion_planner_amd import _abi
    lib = _abi.load()

    def setk(mfma=0, kys=0, lb=0, ba2=0, mbw=0, planar=0, pin=0):
        lib.ffmp_set_tuning(_abi.TUNE_CONV_MFMA, mfma)
        lib.ffmp_set_tuning(_abi.TUNE_CONV_KYS, kys)
        lib.ffmp_set_tuning(_abi.TUNE_CONV_LB, lb)
        lib.ffmp_set_tuning(_abi.TUNE_CONV_BA2, ba2)
        lib.ffmp_set_tuning(_abi.TUNE_CONV_MBW, mbw)
        lib.ffmp_set_tuning(_abi.TUNE_CONV_PLANAR, planar)
        lib.ffmp_set_tuning(_abi.TUNE_CONV_PIN, pin)
    yield setk
    setk()


@pytest.mark.parametrize("B,H,W,C,K,N,pad,dx", [
    (2, 69, 69, 32, 32, 64, 0, 1),    # conv2 (row-ring; LB route)
    (2, 38, 38, 64, 32, 32, 31, 1),   # the padded data-gradient form (one channel block: KYS 4)
    (2, 100, 85, 32, 32, 32, 0, 16),  # conv1 folded (one channel block, dx = 16)
    (3, 38, 38, 64, 8, 64, 0, 1),     # conv3 (small-image kernel)
    (2, 12, 12, 64, 2, 64, 1, 1), (5, 33, 70, 32, 2, 64, 0, 1), (2, 40, 45, 32, 5, 32, 0, 1)])
def test_conv_launch_variants_match_float64(conv_knobs, B, H, W, C, K, N, pad, dx):
    """Every launch variant of the forward (FFMP_TUNE_CONV_MFMA 16 / 32, FFMP_TUNE_CONV_KYS 1 / 2 / 4,
    FFMP_TUNE_CONV_LB, FFMP_TUNE_CONV_BA2, FFMP_TUNE_CONV_MBW 1-4, FFMP_TUNE_CONV_PLANAR, FFMP_TUNE_CONV_PIN) against float64 within the forward's tolerance; the variants that keep the
    32x32x16 accumulation order (kernel rows per ring step, B through LDS) bit-identical to the default."""
    g = torch.Generator(device=DEV).manual_seed(B + H + K + pad)
    xb = torch.randn((B, H, W, C), device=DEV, generator=g).to(torch.bfloat16)
    KW = 2 if dx > 1 else K
    w = torch.randn((N, C, K, KW), device=DEV, generator=g) / (C * K * KW) ** 0.5
    bias = torch.randn(N, device=DEV, generator=g) * 0.1
    wp = pack_weight(w)
    x64 = xb.double().permute(0, 3, 1, 2)
    w64 = wp.double().permute(2, 3, 0, 1)
    with torch.backends.cudnn.flags(enabled=False):
        ref = F.conv2d(x64, w64, bias.double(), padding=pad, dilation=(1, dx)).permute(0, 2, 3, 1)
        absref = F.conv2d(x64.abs(), w64.abs(), padding=pad, dilation=(1, dx)).permute(0, 2, 3, 1)
    conv_knobs(32, 1, 0)
    base = conv2d_nhwc(xb, wp, bias, pad=pad, dx=dx)
    variants = [  # (mfma, kys, lb, ba2, mbw, planar, pin)
        (32, 1, 0, 0, 0, 0, 0), (32, 2, 0, 0, 0, 0, 0), (32, 4, 0, 0, 0, 0, 0), (32, 1, 1, 0, 0, 0, 0),
        (32, 1, 0, 1, 0, 0, 0), (32, 1, 0, 2, 0, 0, 0), (32, 1, 0, 1, 3, 0, 0), (32, 1, 0, 2, 3, 0, 0),
        (32, 1, 0, 0, 1, 0, 0), (32, 1, 0, 0, 2, 0, 0), (32, 1, 0, 0, 3, 0, 0), (32, 1, 0, 0, 4, 0, 0),
        (32, 1, 0, 0, 0, 1, 0), (32, 1, 0, 0, 1, 1, 0), (32, 1, 0, 0, 3, 1, 0), (32, 1, 0, 0, 4, 1, 0),
        (32, 1, 0, 0, 0, 0, 1), (32, 1, 0, 0, 3, 0, 1), (32, 1, 0, 0, 4, 0, 1),
        (16, 1, 0, 0, 0, 0, 0), (16, 4, 0, 0, 0, 0, 0), (0, 0, 0, 0, 0, 0, 0)]
    for mfma, kys, lb, ba2, mbw, planar, pin in variants:
        conv_knobs(mfma, kys, lb, ba2, mbw, planar, pin)
        for wk in (wp, frag_order(wp)):
            y = conv2d_nhwc(xb, wk, bias, pad=pad, dx=dx)
            err = (y.double() - ref).abs()
            bad = err > 5e-5 * absref + 1e-6
            assert not bool(bad.any()), (mfma, kys, lb, ba2, mbw, planar, pin, int(bad.sum()), float(err.max()))
            if mfma in (0, 32):  # the default forward keeps 32x32x16
                assert torch.equal(y, base), (mfma, kys, lb, ba2, mbw, planar, pin)


@pytest.mark.parametrize("mfma", [16, 32])
def test_dgrad_and_wgrad_mfma_shapes_match_float64(conv_knobs, mfma):
    """The samples-as-M data gradient and the weight gradient on both MFMA shapes (conv2's shapes at a
    small batch, and the folded conv1's weight gradient) against float64."""
    from flow_field_based_motion_planner_amd.conv_mfma import conv2d_dgrad_nhwc, conv2d_wgrad_nhwc, pack_weight_dgrad_bm
    conv_knobs(mfma, 0, 0)
    g0 = torch.Generator(device=DEV).manual_seed(mfma)
    g = torch.randn((33, 38, 38, 64), device=DEV, generator=g0).to(torch.bfloat16)
    w = torch.randn((64, 32, 32, 32), device=DEV, generator=g0) / 181.0
    dx = conv2d_dgrad_nhwc(g, pack_weight_dgrad_bm(w), out_dtype=torch.float32)
    g64, w64 = g.double().permute(0, 3, 1, 2), w.to(torch.bfloat16).double()
    with torch.backends.cudnn.flags(enabled=False):
        ref = torch.nn.grad.conv2d_input((33, 32, 69, 69), w64, g64).permute(0, 2, 3, 1)
        absref = torch.nn.grad.conv2d_input((33, 32, 69, 69), w64.abs(), g64.abs()).permute(0, 2, 3, 1)
    assert not bool(((dx.double() - ref).abs() > 5e-5 * absref + 1e-6).any())
    for (B, H, W, C, KH, KW, N, d) in [(3, 69, 69, 32, 32, 32, 64, 1), (2, 100, 85, 32, 32, 2, 32, 16),
                                       (2, 20, 22, 32, 6, 4, 32, 1)]:
        x = torch.randn((B, H, W, C), device=DEV, generator=g0).to(torch.bfloat16)
        gy = torch.randn((B, H - KH + 1, W - (KW - 1) * d, N), device=DEV, generator=g0).to(torch.bfloat16)
        dw = conv2d_wgrad_nhwc(gy, x, KH, KW, dx=d)
        x64, gy64 = x.double().permute(0, 3, 1, 2), gy.double().permute(0, 3, 1, 2)
        with torch.backends.cudnn.flags(enabled=False):
            rw = torch.nn.grad.conv2d_weight(x64, (N, C, KH, KW), gy64, dilation=(1, d)).permute(2, 3, 0, 1)
            aw = torch.nn.grad.conv2d_weight(x64.abs(), (N, C, KH, KW), gy64.abs(), dilation=(1, d)).permute(2, 3, 0, 1)
        assert not bool(((dw.double() - rw).abs() > 5e-5 * aw + 1e-6).any()), (mfma, B, H, KH)


@pytest.mark.parametrize("wgdma", [1, 2, 3, 4])
def test_wgrad_dma_stages_match_float64(wgdma):
    """The weight gradient with LDS-DMA double-buffered stages (FFMP_TUNE_CONV_WGDMA 1, 2 = with the
    k-step prefetch, 4 = conv2's shape at 4 taps per wave) and without them (3) against float64: conv2's shape (64-channel g rows swizzled), conv3's (64-channel x
    rows swizzled too), the folded conv1's and a ragged one (partial last stage, batch chunks)."""
    from flow_field_based_motion_planner_amd import _abi
    from flow_field_based_motion_planner_amd.conv_mfma import conv2d_wgrad_nhwc
    lib = _abi.load()
    prev = lib.ffmp_set_tuning(_abi.TUNE_CONV_WGDMA, wgdma)
    try:
        g0 = torch.Generator(device=DEV).manual_seed(100 + wgdma)
        for (B, H, W, C, KH, KW, N, d) in [(3, 69, 69, 32, 32, 32, 64, 1), (3, 38, 38, 64, 8, 8, 64, 1),
                                           (2, 100, 85, 32, 32, 2, 32, 16), (5, 20, 22, 32, 6, 4, 32, 1)]:
            x = torch.randn((B, H, W, C), device=DEV, generator=g0).to(torch.bfloat16)
            gy = torch.randn((B, H - KH + 1, W - (KW - 1) * d, N), device=DEV, generator=g0).to(torch.bfloat16)
            dw = conv2d_wgrad_nhwc(gy, x, KH, KW, dx=d, chunks=2)
            x64, gy64 = x.double().permute(0, 3, 1, 2), gy.double().permute(0, 3, 1, 2)
            with torch.backends.cudnn.flags(enabled=False):
                rw = torch.nn.grad.conv2d_weight(x64, (N, C, KH, KW), gy64, dilation=(1, d)).permute(2, 3, 0, 1)
                aw = torch.nn.grad.conv2d_weight(x64.abs(), (N, C, KH, KW), gy64.abs(), dilation=(1, d)).permute(2, 3, 0, 1)
            bad = (dw.double() - rw).abs() > 5e-5 * aw + 1e-6
            assert not bool(bad.any()), (wgdma, B, H, C, KH, N, int(bad.sum()))
    finally:
        lib.ffmp_set_tuning(_abi.TUNE_CONV_WGDMA, prev)
