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
    ring = _abi.SeamlessRing(DEV, (7, 48, 48), 3)  # may itself draw pooled pieces of earlier tests
    before = lib.ffmp_ring_pool_bytes(DEV)
    stride = ring.slot_stride
    del ring
    gc.collect()
    pooled = lib.ffmp_ring_pool_bytes(DEV)
    assert pooled == before + 3 * stride
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


def test_rebuild_keep_old_then_revert_or_keep():
    """rebuild(keep_old=True) leaves the old ring whole (its replaced slots keep their bytes);
    revert() makes it current again and drop_previous() releases it; pieces of the released
    ring reach the pool."""
    lib = _abi.load()
    ring = _abi.SeamlessRing(DEV, (3, 40, 40), 4)
    _fill(ring.tensor, 4)
    old_t = ring.tensor
    ring.rebuild(0b0010, keep_old=True)  # replace slot 1
    new_t = ring.tensor
    assert new_t.data_ptr() != old_t.data_ptr()
    assert float(new_t[2].min()) == 3.0 and float(new_t[0].max()) == 1.0  # kept slots shared
    new_t[1].fill_(-5.0)
    torch.cuda.synchronize()
    assert float(old_t[1].min()) == 2.0 and float(old_t[1].max()) == 2.0  # old slot 1 untouched
    new_t[2].fill_(8.0)  # a kept slot is the same memory in both rings
    torch.cuda.synchronize()
    assert float(old_t[2].min()) == 8.0
    pooled = lib.ffmp_ring_pool_bytes(DEV)
    ring.revert()
    assert ring.tensor.data_ptr() == old_t.data_ptr() and ring.info()["reverts"] == 1
    del new_t
    gc.collect()
    assert lib.ffmp_ring_pool_bytes(DEV) == pooled + ring.slot_stride  # the new slot-1 piece
    ring.rebuild(0b0001, keep_old=True)
    ring.drop_previous()
    del old_t
    gc.collect()
    assert lib.ffmp_ring_pool_bytes(DEV) >= pooled + ring.slot_stride  # old slot 0 freed (new one drawn)
    t = ring.tensor
    t[0].fill_(4.0)
    torch.cuda.synchronize()
    assert torch.equal(t[4], t[0]) and float(t[1].max()) == 2.0
    with pytest.raises(RuntimeError):
        ring.revert()


def test_repair_keeps_a_working_ring():
    """_repair_slots with every slot declared slow rebuilds, times, and keeps or reverts; either
    way the env still matches the contiguous layout bit for bit."""
    from flow_field_based_motion_planner_amd.config import FFMPConfig
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    cfg = FFMPConfig(grid=64, n_obst=6, n_beams=16, moving=True, max_steps=6, seed=9)
    a = FFMPVec(12, cfg, device="cuda:0", frame_window=2)
    b = FFMPVec(12, cfg, device="cuda:0", frame_window=4, seamless=True, autotune=False)
    b.SLOW_SLOT = -1.0  # every slot is "slow": forces the rebuild + keep/revert path
    b._repair_slots()
    hist = b.ring_meta["repair"]
    assert b._ring.info()["rebuilds"] >= 1 and len(hist) >= 2
    a.reset()
    b.reset()
    g = torch.Generator().manual_seed(1)
    for _ in range(10):
        act = torch.randint(0, 28, (12,), generator=g).to("cuda:0")
        oa, ob = a.step(act)[0], b.step(act)[0]
        assert torch.equal(oa["state_m"], ob["state_m"]) and torch.equal(oa["potential"], ob["potential"])


def test_repair_survives_a_failed_rebuild():
    """A slot rebuild that fails (out of HBM with several ranks on one device: bench.py --gpus 4
    rehearsed on one GPU, profiles/r04n_launcher.txt) leaves the current ring in place; the repair
    records the reason and the env still matches the contiguous layout bit for bit."""
    from flow_field_based_motion_planner_amd import _abi
    from flow_field_based_motion_planner_amd.config import FFMPConfig
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    cfg = FFMPConfig(grid=64, n_obst=6, n_beams=16, moving=True, max_steps=6, seed=9)
    a = FFMPVec(12, cfg, device="cuda:0", frame_window=2)
    b = FFMPVec(12, cfg, device="cuda:0", frame_window=4, seamless=True, autotune=False)
    handle = b._ring.handle

    def no_memory(*args, **kw):
        raise _abi.FFMPBackendError("ffmp_ring_rebuild failed (rc=-2): out of memory (test)")

    b._ring.rebuild = no_memory
    b.SLOW_SLOT = -1.0
    b._repair_slots()
    assert b._ring.handle == handle and b._ring.info()["rebuilds"] == 0
    assert "out of memory" in b.ring_meta["repair"][-1]["skipped"]
    a.reset()
    b.reset()
    g = torch.Generator().manual_seed(2)
    for _ in range(10):
        act = torch.randint(0, 28, (12,), generator=g).to("cuda:0")
        oa, ob = a.step(act)[0], b.step(act)[0]
        assert torch.equal(oa["state_m"], ob["state_m"]) and torch.equal(oa["potential"], ob["potential"])


def test_partner_relocation_keeps_a_consistent_env():
    """With every pairing probe declared slow, FFMPVec re-allocates the potential plane's arena and
    re-pairs a ring against it (up to PARTNER_TRIES times), keeping the best pair; the kept arena
    and ring still give the contiguous layout's observations bit for bit."""
    from flow_field_based_motion_planner_amd.config import FFMPConfig
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    free, _ = torch.cuda.mem_get_info(DEV)
    if free < (80 << 30):
        pytest.skip("needs ~80 GiB of free HBM")

    class Picky(FFMPVec):
        PAIR_FAST_GBS = 1e9  # nothing is fast enough: every try runs
        REPAIR_ROUNDS = 0    # (a slot rebuild would report only its new pieces' probes)

    cfg = FFMPConfig(grid=256, n_obst=8, n_beams=32, moving=True, max_steps=5, seed=17)
    n = 8192  # 2 GiB frame slots (1 GiB pieces, probed) + 2 GiB potential plane
    tune = {"shape": [8192, _abi.RASTER_NT], "shape_newest": [8192, _abi.RASTER_NT], "fused": False}
    b = Picky(n, cfg, device="cuda:0", frame_window=3, seamless=True, tuning=tune)
    meta = b.ring_meta
    assert b.ring == "seamless" and len(meta["partner_tries"]) >= 2, meta
    assert meta["pair_gbs_max"] == max(meta["partner_tries"])
    a = FFMPVec(n, cfg, device="cuda:0", frame_window=2, autotune=False)
    a.reset()
    b.reset()
    g = torch.Generator().manual_seed(3)
    for _ in range(5):
        act = torch.randint(0, 28, (n,), generator=g).to("cuda:0")
        oa, ob = a.step(act)[0], b.step(act)[0]
        assert torch.equal(oa["state_m"], ob["state_m"]) and torch.equal(oa["potential"], ob["potential"])


def test_pair_probe_stays_inside_a_compact_partner_and_rebuild_keeps_the_scale():
    """Compact ring (uint8 slots beside a binary16 plane of twice the bytes) whose last piece's
    probe length is not a multiple of 256 float4s (G = 100): the two-stream pairing probe must not
    write past the partner (a guard band after it keeps its bytes), and a rebuild pairs with the
    ratio fixed at create (slots of ~2.1 GiB round up to a 3 GiB stride, from which the ratio would
    have been guessed as 1)."""
    free, _ = torch.cuda.mem_get_info(DEV)
    if free < (40 << 30):
        pytest.skip("needs ~40 GiB of free HBM")
    G = 100
    n = 225486                      # 2.1 GiB uint8 slot; partner 4.2 GiB
    slot = n * G * G
    pbytes = 2 * slot
    last = (pbytes - 4 * (1 << 30)) // 2  # slot bytes of the last 1 GiB piece with partner beside them
    assert last >= (64 << 20) and (last // 16) % 256 != 0
    guard = 1 << 20
    buf = torch.zeros(pbytes + guard, dtype=torch.uint8, device=f"cuda:{DEV}")
    buf[pbytes:].fill_(0xA5)
    partner = buf[:pbytes]
    ring = _abi.SeamlessRing(DEV, (n, G, G), 3, bits=8, partner=partner)
    torch.cuda.synchronize()
    info = ring.info()
    assert info["pair_scale"] == 2 and info["pieces"] == 9 and info["pair_probes"] >= 3, info
    assert bool((buf[pbytes:] == 0xA5).all()), "pairing probe wrote past the partner"
    ring.rebuild(0b100, partner=partner)
    torch.cuda.synchronize()
    assert ring.info()["pair_scale"] == 2
    assert bool((buf[pbytes:] == 0xA5).all()), "rebuild probe wrote past the partner"
    t = ring.tensor
    t[3, :4].fill_(7)  # the alias slot still maps slot 0
    torch.cuda.synchronize()
    assert int(t[0, :4].sum()) == 7 * 4 * G * G


def test_pool_trim_gives_memory_back_and_later_rings_see_their_writes():
    """ffmp_ring_pool_trim: the pooled pieces' memory goes back to the device (every mapping of
    them unmapped, the address ranges kept reserved), and rings built afterwards — at fresh
    addresses — read back exactly what kernels and host copies wrote (the stale-resolution hazard
    of a REUSED address, tools/ring_reuse_probe.hip, cannot arise: no address is reused)."""
    lib = _abi.load()
    _abi.ring_pool_trim(DEV, 0)
    assert lib.ffmp_ring_pool_bytes(DEV) == 0
    shape = (64, 1024, 1024)  # 256 MiB slots, one piece each
    rings = [_abi.SeamlessRing(DEV, shape, 4) for _ in range(2)]
    rings[1].rebuild(0b0011)  # the replaced pieces stay held by the old ring until it is dropped
    rings[1].drop_previous()
    stride = rings[0].slot_stride
    for r in rings:
        _fill(r.tensor, 4)
    del r
    rings = None
    gc.collect()
    pooled = lib.ffmp_ring_pool_bytes(DEV)
    assert pooled >= 8 * stride
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(DEV)
    released = _abi.ring_pool_trim(DEV, 0)
    free1, _ = torch.cuda.mem_get_info(DEV)
    assert released == pooled and lib.ffmp_ring_pool_bytes(DEV) == 0
    assert free1 - free0 >= 0.95 * released, (free0, free1, released)
    # keep_bytes: the first pieces up to it stay pooled
    a = _abi.SeamlessRing(DEV, shape, 3)
    del a
    gc.collect()
    assert _abi.ring_pool_trim(DEV, stride) == 2 * stride and lib.ffmp_ring_pool_bytes(DEV) == stride
    # new rings after the release: kernel writes, host-to-device copies and the alias all land
    for k in range(3):
        r = _abi.SeamlessRing(DEV, shape, 3)
        t = r.tensor
        for i in range(3):
            t[i].fill_(float(10 * k + i))
        torch.cuda.synchronize()
        host = t[:4].cpu()  # the D2H copy is what returned an old ring's bytes at a reused address
        for i in range(3):
            assert float(host[i].min()) == float(host[i].max()) == float(10 * k + i), (k, i)
        assert torch.equal(host[3], host[0])
        pattern = torch.arange(shape[1] * shape[2], dtype=torch.float32).view(shape[1:])
        t[1, 5].copy_(pattern)
        torch.cuda.synchronize()
        assert torch.equal(t[1, 5].cpu(), pattern)
        del t, r, host
        gc.collect()
    _abi.ring_pool_trim(DEV, 0)


def test_closing_one_instance_keeps_the_others_pairing_references():
    """trimming the pool on close had erased every instance's pairing references (the
    best probe per partner plane that a later slot-repair rebuild is judged against).  Now an
    instance forgets only the references of the planes it frees."""
    from flow_field_based_motion_planner_amd.config import preset
    from flow_field_based_motion_planner_amd.vec_env import FFMPVec
    lib = _abi.load()
    gc.collect()  # instances earlier tests dropped without close() forget their references here
    # rings the earlier tests built against bare partner tensors left references keyed by addresses
    # torch hands out again (forgetting them before freeing a plane is the caller's job: ffmp.h)
    _abi.ring_pair_forget(0)
    r0 = lib.ffmp_ring_pair_refs(0)
    assert r0 == 0
    a = FFMPVec(4096, preset("C2", seed=1), device="cuda:0", autotune=False)
    assert a.ring == "seamless"
    ra = lib.ffmp_ring_pair_refs(0)
    assert ra > r0
    b = FFMPVec(4096, preset("C2", seed=2), device="cuda:0", autotune=False)
    assert lib.ffmp_ring_pair_refs(0) > ra
    b.close()
    assert lib.ffmp_ring_pair_refs(0) == ra
    a.close()
    assert lib.ffmp_ring_pair_refs(0) == r0
    # an instance dropped without close() forgets its references when it is collected
    c = FFMPVec(4096, preset("C2", seed=3), device="cuda:0", autotune=False)
    assert lib.ffmp_ring_pair_refs(0) > r0
    del c
    gc.collect()
    assert lib.ffmp_ring_pair_refs(0) == r0
