"""The 12-channel BEV option (src/train.py:66 "(occupancy(MONO) + flow(RGB)) * series(3 steps)",
src/gym_ffmp/envs/ffmp.py:16) on the CPU: the stated RGB flow encoding of the oracle
(oracle.ffmp_oracle.bev_image, include/ffmp.h ffmp_bev_image), the C entry point's argument checks
(no launch), and the MFMA fold of a 12-channel conv1.  The reference's own RGB encoding lived in BEV
nodes outside its repository: parity of the colours is unpinned against the reference; the
occupancy channel and the flow planes they encode are the pinned raster's."""
import ctypes as C

import numpy as np
import pytest
import torch

from flow_field_based_motion_planner_amd import _abi
from oracle.ffmp_oracle import bev_image

F32 = np.float32


def test_encoding_fixed_points_and_inverse():
    vmax = 1.2
    v = F32(vmax)
    fx = np.array([0.0, vmax, -vmax, 0.5 * vmax, -0.25, 2 * vmax, 0.3], dtype=F32)
    fy = np.array([0.0, 0.0, 0.0, -0.5 * vmax, 0.7, 0.0, -0.4], dtype=F32)
    occ = np.array([0, 255, 0, 255, 0, 255, 0], dtype=F32)
    img = bev_image(occ.reshape(1, 1, -1), np.stack([fx, fy]).reshape(1, 2, 1, -1), vmax)[0, :, 0]
    assert img.dtype == np.float32 and img.shape == (4, 7)
    assert np.array_equal(img[0], occ)
    assert img[1:, 0].tolist() == [128.0, 128.0, 0.0]     # no motion: rint(127.5) = 128 (half to even)
    assert img[1:, 1].tolist() == [255.0, 128.0, 255.0]   # +vmax along x, full speed
    assert img[1:, 2].tolist() == [0.0, 128.0, 255.0]     # -vmax
    assert img[1:, 5].tolist() == [255.0, 128.0, 255.0]   # beyond vmax: clamped
    # every channel is an integer in [0, 255], and the axis channels invert to within half a step
    assert np.array_equal(img, np.rint(img)) and img.min() >= 0 and img.max() <= 255
    inner = np.abs(fx) <= v
    back = (img[1] - F32(127.5)) / F32(127.5) * v
    assert np.all(np.abs(back - fx)[inner] <= v / 255 + 1e-6)
    speed = np.hypot(fx, fy)
    assert np.all(np.abs(img[3] / 255 * v - np.minimum(speed, v)) <= v / 510 + 1e-6)


def test_encoding_is_monotone_and_symmetric():
    vmax = 0.5
    x = np.linspace(-vmax, vmax, 2001, dtype=F32)
    img = bev_image(np.zeros((1, 1, x.size), F32), np.stack([x, -x]).reshape(1, 2, 1, -1), vmax)[0, :, 0]
    assert np.all(np.diff(img[1]) >= 0) and np.all(np.diff(img[2]) <= 0)
    # R(v) + R(-v) = 255 up to the half-to-even rounding of exact halves (v = 0: 128 + 128)
    assert np.all(np.abs(img[1] + img[1][::-1] - 255) <= 1)
    assert np.array_equal(img[3], img[3][::-1])


@pytest.fixture(scope="module")
def lib():
    return _abi.load()


def test_entry_point_argument_checks_no_gpu(lib):
    buf = (C.c_float * 64)()
    p = C.cast(buf, C.c_void_p).value
    f = lib.ffmp_bev_image
    assert f(0, 0, p, 16, p, 16, 1.0, p, 64, None) == 0            # n = 0: nothing to launch
    assert f(-1, 0, p, 16, p, 16, 1.0, p, 64, None) == -1
    assert f(1, 0, p, 16, p, 16, 0.0, p, 64, None) == -1 and b"vmax" in lib.ffmp_last_error()
    assert f(1, 0, p, 16, p, 16, float("inf"), p, 64, None) == -1
    assert f(1, 0, p, 16, p, 16, 1.0, p, 63, None) == -1 and b"out_env_stride" in lib.ffmp_last_error()
    assert f(1, 0, p, 15, p, 16, 1.0, p, 64, None) == -1
    assert f(1, 2, p, 16, p, 16, 1.0, p, 64, None) == -1 and b"compact" in lib.ffmp_last_error()
    assert f(1, 0, None, 16, p, 16, 1.0, p, 64, None) == -1 and b"NULL" in lib.ffmp_last_error()


def test_twelve_channel_conv1_folds_onto_the_mfma_kernel():
    """conv1 of Network(input_channels=12) pads to 16 channels and folds F = 2 kernel columns into
    32 channels, like 3 -> 4 channels at F = 8: the library's launch checks accept both launches."""
    from flow_field_based_motion_planner_amd import conv_mfma
    assert conv_mfma.fold_channels(12) == 16 and conv_mfma.fold_channels(3) == 4 and conv_mfma.fold_channels(2) == 2
    c1 = torch.nn.Conv2d(12, 32, kernel_size=32)
    assert conv_mfma.fold_supported(c1, (256, 12, 100, 100))
    assert not conv_mfma.fold_supported(torch.nn.Conv2d(17, 32, kernel_size=32))
