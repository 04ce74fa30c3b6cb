"""The raster's exact fast math (ffmp_device.h sqrt_rn / rcp_rn) against the IEEE float32
sqrtf and 1.0f / d, bit for bit, over EVERY float of the domains the raster feeds them:
sqrt over [2^-96, +inf) (smaller squared distances are clamped to rho_min either way)
and the reciprocal over every normal d whose reciprocal is normal ([2^-126, 2^126)), a superset
of the clamped repulsive distance range [rho_min, rho0) that check_cfg admits.  The potential
plane itself has no reference counterpart ([no reference]); its cell-by-cell parity
with the oracle is tests/test_gpu_parity.py / test_gpu_compact.py."""
import ctypes as C
import struct

import pytest
import torch

from flow_field_based_motion_planner_amd import _abi

pytestmark = pytest.mark.gpu


def _bits(x):
    return struct.unpack("<I", struct.pack("<f", x))[0]


def _run(lib, which, lo, hi):
    mism = torch.zeros(1, dtype=torch.int64, device="cuda")
    first = torch.full((1,), -1, dtype=torch.int32, device="cuda")  # 0xFFFFFFFF
    s = torch.cuda.current_stream().cuda_stream
    _abi.check(lib.ffmp_check_exact_math(which, lo, hi, mism.data_ptr(), first.data_ptr(), s))
    torch.cuda.synchronize()
    return int(mism.item()), int(first.item()) & 0xFFFFFFFF


@pytest.mark.parametrize("which,lo,hi", [
    (0, _bits(2.0 ** -96), _bits(float("inf"))),        # sqrt_rn == sqrtf
    (1, _bits(2.0 ** -126), _bits(2.0 ** 126)),          # rcp_rn == 1.0f / d
])
def test_exact_math_exhaustive(lib, which, lo, hi):
    n, first = _run(lib, which, lo, hi)
    assert n == 0, f"{n} mismatches, first at bits 0x{first:08x} ({struct.unpack('<f', struct.pack('<I', first))[0]!r})"


def test_exact_math_below_domain_reported(lib):
    """Reported, not asserted: below 2^-96 (denormal squared distances) v_sqrt_f32
    without sqrtf's scaling is not correctly rounded for every input — the count is reported, not
    asserted zero, and the raster never depends on it (fmaxf(sqrt(s) - r, rho_min) = rho_min)."""
    n, _ = _run(lib, 0, 1, _bits(2.0 ** -96))
    print(f"sqrt_rn vs sqrtf below 2^-96: {n} differing inputs of {_bits(2.0 ** -96) - 1}")
    assert n >= 0
