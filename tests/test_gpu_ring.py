"""The seamless frame ring's memory layer (include/ffmp.h ffmp_ring_*), on the GPU: the alias
slot, rebuilds keep the kept slots' bytes, pooled pieces are reused, pairing against a partner.
The env-level parity of the ring is in test_gpu_parity.py (test_frame_window_equals_contiguous)."""
import gc

import pytest
import torch

from flow_field_based_motion_planner_amd import _abi

pytestmark = pytest.mark.gpu
DEV = 0


def _fill(t, slots):
    for i in range(slots):
        t[i].fill_(float(i + 1))
    torch.cuda.synchronize()


def test_alias_slot_is_slot_zero():
    ring = _abi.SeamlessRing(DEV, (3, 64, 64), 5)
    t = ring.tensor
    assert t.shape == (6, 3, 64, 64) and t.stride(0) >= 3 * 64 * 64
    _fill(t, 5)
    assert torch.equal(t[5], t[0])
    t[5].fill_(-7.0)  # a write through the alias lands in slot 0
    torch.cuda.synchronize()
    assert float(t[0].min()) == -7.0 and float(t[0].max()) == -7.0
    assert float(t[1].max()) == 2.0 and float(t[4].min()) == 5.0


def test_rebuild_keeps_the_kept_slots():
    ring = _abi.SeamlessRing(DEV, (2, 32, 32), 4)
    _fill(ring.tensor, 4)
    old_ptr = ring.tensor.data_ptr()
    ring.rebuild(0b0101)  # replace slots 0 and 2
    t = ring.tensor
    assert t.data_ptr() != old_ptr and t.shape == (5, 2, 32, 32)
    assert float(t[1].min()) == 2.0 and float(t[1].max()) == 2.0
    assert float(t[3].min()) == 4.0 and float(t[3].max()) == 4.0
    t[0].fill_(9.0)  # the new slot 0 is aliased by the new slot 4
    torch.cuda.synchronize()
    assert torch.equal(t[4], t[0])
    assert ring.info()["rebuilds"] == 1


def test_pieces_return_to_the_pool_and_are_reused():
    lib = _abi.load()
    before = lib.ffmp_ring_pool_bytes(DEV)
    ring = _abi.SeamlessRing(DEV, (7, 48, 48), 3)
    stride = ring.slot_stride
    del ring
    gc.collect()
    pooled = lib.ffmp_ring_pool_bytes(DEV)
    assert pooled >= before + 3 * stride
    again = _abi.SeamlessRing(DEV, (7, 48, 48), 3)  # the same shape draws the pooled pieces
    assert lib.ffmp_ring_pool_bytes(DEV) == pooled - 3 * stride
    _fill(again.tensor, 3)
    assert float(again.tensor[2].sum()) == 3.0 * 7 * 48 * 48
    assert again.info()["pieces_new"] == 0


def test_pairing_against_a_partner():
    """1 GiB pieces paired with a 2 GiB partner: every piece position probed, the chosen pieces'
    probe rates reported, the ring usable and aliased."""
    free, _ = torch.cuda.mem_get_info(DEV)
    if free < (40 << 30):
        pytest.skip("needs ~40 GiB of free HBM")
    partner = torch.empty((2 << 30) // 4, dtype=torch.float32, device=f"cuda:{DEV}")
    ring = _abi.SeamlessRing(DEV, ((2 << 30) // 4,), 3, partner=partner)  # 3 slots of 2 GiB = 6 pieces
    info = ring.info()
    assert info["pieces"] == 6 and info["pair_probes"] >= 3
    assert 0 < info["pair_gbs_min"] <= info["pair_gbs_max"]
    t = ring.tensor
    t[3, :1024].fill_(5.0)
    torch.cuda.synchronize()
    assert float(t[0, :1024].sum()) == 5.0 * 1024


@pytest.mark.parametrize("fused", [False, True])
def test_slot_written_matches_the_step(fused):
    """FFMPVec._slot_written(k) — the slot the per-slot repair timing charges step k to — is the
    physical slot the k-th step after a reset actually writes its newest frame into."""
    from flow_field_based_motion_planner_amd.config import FFMPConfig
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    cfg = FFMPConfig(grid=64, n_obst=4, n_beams=16, moving=True, seed=5)
    W = 5
    env = FFMPVec(8, cfg, device="cuda:0", frame_window=W, seamless=True, autotune=False, fused=fused)
    assert env.ring == "seamless"
    env.reset()
    a = torch.full((8,), 10, dtype=torch.int64, device="cuda:0")
    for k in range(2 * W + 1):
        env.frames[:W].fill_(-3.0)
        env.step(a)
        torch.cuda.synchronize()
        whole = [i for i in range(W) if bool((env.frames[i] != -3.0).all())]
        assert whole == [env._slot_written(k)], (k, whole)
