"""Host-side checks of conv_mfma's weight-pack cache and ReLU backward (CPU tensors; the kernels
themselves are covered by tests/test_gpu_conv_mfma.py)."""
import torch

from flow_field_based_motion_planner_amd import conv_mfma


def test_pack_cache_reuses_until_the_weight_changes():
    conv = torch.nn.Conv2d(32, 64, kernel_size=4)
    w = conv.weight
    a = conv_mfma.packed(w, "fwd", conv_mfma.pack_weight)
    assert conv_mfma.packed(w, "fwd", conv_mfma.pack_weight) is a
    assert torch.equal(a, conv_mfma.pack_weight(w))
    b = conv_mfma.packed(w, "dgrad_bm", conv_mfma.pack_weight_dgrad_bm)
    assert b is not a and torch.equal(b, conv_mfma.pack_weight_dgrad_bm(w))
    # an optimizer step (in-place update) invalidates every pack of the weight
    opt = torch.optim.SGD(conv.parameters(), lr=0.1)
    conv(torch.randn(2, 32, 8, 8)).sum().backward()
    opt.step()
    a2 = conv_mfma.packed(w, "fwd", conv_mfma.pack_weight)
    assert a2 is not a and torch.equal(a2, conv_mfma.pack_weight(w))
    assert not torch.equal(a2, a)
    # so does load_state_dict (copy_ into the parameter)
    conv.load_state_dict({k: torch.zeros_like(v) for k, v in conv.state_dict().items()})
    a3 = conv_mfma.packed(w, "fwd", conv_mfma.pack_weight)
    assert a3 is not a2 and int(a3.float().abs().sum()) == 0


def test_fused_optimizer_step_invalidates_packs():
    """torch's fused Adam writes parameters without bumping _version: track_optimizer's
    step post-hook must bump it, or the cached packs would outlive every update."""
    conv = torch.nn.Conv2d(32, 64, kernel_size=4)
    w = conv.weight
    opt = torch.optim.Adam(conv.parameters(), lr=0.1, fused=True)
    conv(torch.randn(2, 32, 8, 8)).sum().backward()
    v0 = w._version
    opt.step()
    assert w._version == v0  # the hazard itself: the fused step leaves the version alone
    a = conv_mfma.packed(w, "fwd", conv_mfma.pack_weight)
    conv_mfma.track_optimizer(opt)
    for _ in range(2):
        conv(torch.randn(2, 32, 8, 8)).sum().backward()
        opt.step()
        a2 = conv_mfma.packed(w, "fwd", conv_mfma.pack_weight)
        assert a2 is not a and torch.equal(a2, conv_mfma.pack_weight(w)) and not torch.equal(a2, a)
        a = a2


def test_brain_tracks_its_optimizer():
    """Brain's Adam carries the version-bumping hook (learner.py)."""
    from flow_field_based_motion_planner_amd.learner import Brain
    import inspect
    assert "track_optimizer(self.optimizer)" in inspect.getsource(Brain.__init__)


def test_pack_cache_without_attributes_falls_back():
    class NoAttr(torch.Tensor):
        def __setattr__(self, name, value):
            raise AttributeError(name)
    w = torch.randn(64, 32, 2, 2).as_subclass(NoAttr)
    calls = []

    def fn(v):
        calls.append(1)
        return conv_mfma.pack_weight(v.as_subclass(torch.Tensor))
    conv_mfma.packed(w, "fwd", fn)
    conv_mfma.packed(w, "fwd", fn)
    assert len(calls) == 2


def test_relu_backward_matches_mask_multiply():
    torch.manual_seed(0)
    y = torch.relu(torch.randn(3, 5, 6, 64)).to(torch.bfloat16)            # NHWC ReLU output
    y[0, 0, 0, :4] = 0
    gy = torch.randn(3, 64, 5, 6).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g = conv_mfma.relu_masked_nhwc(gy, y)
    ref = (gy.permute(0, 2, 3, 1) * (y > 0)).contiguous()
    assert g.is_contiguous() and g.shape == (3, 5, 6, 64) and g.dtype == torch.bfloat16
    assert torch.equal(g, ref)
    # an fp32 incoming gradient is rounded to bf16 first, as before
    g32 = conv_mfma.relu_masked_nhwc(gy.float(), y)
    assert torch.equal(g32, ref)


def test_frag_order_matches_the_header_index():
    """conv_mfma.frag_order puts weight (ky, kx, o, i) where include/ffmp.h's FFMP_CONV_W_FRAG says."""
    KH, KW, N, Cc = 2, 3, 64, 32
    wp = torch.arange(KH * KW * N * Cc, dtype=torch.float32).view(KH, KW, N, Cc)
    flat = conv_mfma.frag_order(wp).flatten()
    assert flat.shape == wp.flatten().shape
    for ky, kx, o, i in [(0, 0, 0, 0), (1, 2, 63, 31), (0, 1, 33, 9), (1, 0, 5, 17), (1, 1, 40, 24)]:
        idx = ((((ky * KW + kx) * (N // 32) + o // 32) * (Cc // 16) + i // 16) * 2 + (i % 16) // 8) * 256 \
            + (o % 32) * 8 + i % 8
        assert flat[idx] == wp[ky, kx, o, i]


def test_small_route_mirrors_the_library_shapes():
    """The Network's conv3 / conv4 forwards and their data gradients run on the small-image kernel
    (fragment-order weights); conv2 and its transposed form on the row-ring kernel."""
    for h in (38, 31, 24, 17):
        assert conv_mfma.small_route(h, h, 64, 8, 8)
    for hy in (31, 24, 17, 10):
        assert conv_mfma.small_route(hy, hy, 64, 8, 8, pad=7)
    assert not conv_mfma.small_route(69, 69, 32, 32, 32)       # conv2
    assert not conv_mfma.small_route(38, 38, 64, 32, 32, 31)   # conv2's transposed form
    assert not conv_mfma.small_route(100, 69, 32, 32, 2, 0, 16)  # the folded conv1
