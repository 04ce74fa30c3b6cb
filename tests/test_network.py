"""Batched Network (network.py) against the reference Network (src/train.py:231-303) run by
tests/golden/make_golden.py on the same deterministic weights and inputs (golden "network").
CPU: float32 torch on the host (the learner is a torch consumer, not a HIP kernel);
GPU: the same on cuda:0, where MIOpen's convolution algorithms reorder the float32 sums."""
import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd.network import Network
from tests.parity_util import network_inputs, network_weights

# |q| ~ 10; float32 sums over up to 32,768 products per output of conv2
CPU_ATOL, GPU_ATOL, RTOL = 1e-4, 2e-3, 1e-4


def _net(golden, device, coupling="reference"):
    net = Network(2, 28, grid=100, coupling=coupling)
    shapes = [(k, tuple(v)) for k, v in golden["network"]["param_shapes"]]
    assert [(k, tuple(v.shape)) for k, v in net.state_dict().items()] == shapes
    net.load_state_dict({k: torch.from_numpy(v) for k, v in network_weights(shapes).items()})
    return net.to(device).eval()


def _inputs(case, device):
    return [torch.from_numpy(x).to(device) for x in network_inputs(case["batch"], case["seed"])]


def _check(golden, device, atol):
    net = _net(golden, device)
    for case in golden["network"]["cases"]:
        with torch.no_grad():
            q = net(*_inputs(case, device)).cpu().numpy()
        want = np.asarray(case["q"], dtype=np.float32)
        assert q.shape == want.shape
        np.testing.assert_allclose(q, want, rtol=RTOL, atol=atol, err_msg=f"batch {case['batch']}")


def test_reference_outputs_cpu(golden):
    _check(golden, "cpu", CPU_ATOL)


def test_per_sample_coupling_cpu(golden):
    """per_sample == running each sample alone (the reference's B=1 result), and differs from
    the reference coupling at B>1."""
    ref = _net(golden, "cpu")
    per = _net(golden, "cpu", coupling="per_sample")
    case = next(c for c in golden["network"]["cases"] if c["batch"] == 3)
    sm, g, v, t = _inputs(case, "cpu")
    with torch.no_grad():
        batched = per(sm, g, v, t)
        alone = torch.cat([ref(sm[i:i + 1], g[i:i + 1], v[i:i + 1], t[i:i + 1]) for i in range(3)])
        coupled = ref(sm, g, v, t)
    torch.testing.assert_close(batched, alone, rtol=1e-5, atol=1e-4)
    assert not torch.allclose(coupled[1:], alone[1:], atol=1e-3)
    torch.testing.assert_close(coupled[:1], alone[:1], rtol=1e-5, atol=1e-4)


def test_grid_validation():
    with pytest.raises(ValueError):
        Network(grid=64)
    with pytest.raises(ValueError):
        Network(grid=256)
    assert Network(grid=128).fc2.in_features == 64 * 38 * 38


@pytest.mark.gpu
def test_reference_outputs_gpu(golden):
    _check(golden, "cuda:0", GPU_ATOL)


def test_map_channels_options():
    """train.py:66-69's INPUT_CHANNELS options: 2 = [older, newest], 1 = newest, 3 = newest + flow xy."""
    import pytest
    import torch

    from flow_field_based_motion_planner_amd.network import map_channels
    sm = torch.arange(2 * 2 * 4 * 4, dtype=torch.float32).reshape(2, 2, 4, 4)
    fl = -torch.arange(2 * 2 * 4 * 4, dtype=torch.float32).reshape(2, 2, 4, 4)
    assert map_channels(sm, None, 2) is sm
    assert torch.equal(map_channels(sm, None, 1), sm[:, 1:2])
    m3 = map_channels(sm, fl, 3)
    assert m3.shape == (2, 3, 4, 4) and torch.equal(m3[:, 0], sm[:, 1]) and torch.equal(m3[:, 1:], fl)
    u8 = (sm > 10).to(torch.uint8) * 255
    assert map_channels(u8, None, 2).dtype == torch.float32 and torch.equal(map_channels(u8, None, 2), u8.float())
    with pytest.raises(ValueError):
        map_channels(sm, None, 3)
    with pytest.raises(ValueError):
        map_channels(sm, fl, 12)


def test_mfma_support_follows_the_kernels_shape_limits():
    """conv_mfma.supported / fold_supported with the input shape ask the library's own launch checks
    (include/ffmp.h ffmp_conv2d_check, no GPU needed): the reference's G = 100 stack is taken whole;
    64-channel rows over 16 KiB (conv3 at G >= 191), weight-gradient rows under 8 positions (the
    third conv4 at G = 91-97) and a batch over 65,535 are not, so Network keeps F.relu(conv(x))
    for exactly those layers."""
    from flow_field_based_motion_planner_amd import conv_mfma
    c1, c2 = torch.nn.Conv2d(2, 32, 32), torch.nn.Conv2d(32, 64, 32)
    c3, c4 = torch.nn.Conv2d(64, 64, 8), torch.nn.Conv2d(64, 64, 8)
    B = 256
    assert conv_mfma.fold_supported(c1, (B, 2, 100, 100)) and conv_mfma.supported(c2, (B, 32, 69, 69))
    assert conv_mfma.supported(c3, (B, 64, 38, 38))
    assert all(conv_mfma.supported(c4, (B, 64, s, s)) for s in (31, 24, 17))
    assert not conv_mfma.supported(c4, (B, 64, 13, 13))      # G = 96: wgrad output rows of 6
    assert not conv_mfma.supported(c3, (B, 64, 260, 260))    # 64-channel rows of 33 KiB
    assert not conv_mfma.supported(c2, (70000, 32, 69, 69))  # batch over 65,535
    assert not conv_mfma.supported(c2, (B, 64, 69, 69))      # channel mismatch
    assert conv_mfma.supported(c2) and not conv_mfma.supported(c1)  # layer-only form
