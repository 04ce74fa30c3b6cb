"""Host logic and the C ABI without a GPU: the library loads, exports every symbol
include/ffmp.h declares, its struct layout matches the ctypes binding, and the
host-side entry points / argument validation behave (no kernel is launched)."""
import ctypes as C
import json
import math
import os
import re

import numpy as np
import pytest

from flow_field_based_motion_planner_amd import _abi
from flow_field_based_motion_planner_amd.config import (PRESETS, FFMPConfig, beam_table, bytes_per_env_step,
                                                        footprint_offsets, preset)

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "ffmp.h")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(ffmp_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported(lib):
    names = header_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_abi._SIGS), "ctypes binding must cover exactly the header's entry points"


def test_layout_and_version(lib):
    assert lib.ffmp_abi_version() == _abi.ABI_VERSION
    _abi.verify_layout(lib)


@pytest.mark.parametrize("G", [8, 64, 100, 128, 256, 512])
def test_footprint_lib_equals_host(lib, G):
    assert _abi.footprint_from_lib(G, 0.05, 0.13) == footprint_offsets(G)


def test_footprint_other_radii(lib):
    for r in (0.0, 0.05, 0.2, 0.31):
        assert _abi.footprint_from_lib(128, 0.05, r) == footprint_offsets(128, 0.05, r)


def _null_structs():
    return _abi.StateT(), _abi.ObsT(), _abi.OutT()


def test_argument_validation_no_gpu(lib):
    cfg = _abi.make_cfg(FFMPConfig(grid=64, n_obst=4, n_beams=0))
    st, ob, out = _null_structs()
    rc = lib.ffmp_step(C.byref(cfg), 4, 0, None, C.byref(st), C.byref(ob), C.byref(out), None)
    assert rc == -1 and b"NULL" in lib.ffmp_last_error()
    bad = _abi.make_cfg(FFMPConfig(grid=64, n_obst=4, n_beams=0))
    bad.grid = 66
    assert lib.ffmp_raster(C.byref(bad), 1, None, None, C.byref(ob), None) == -3
    assert b"multiple of 4" in lib.ffmp_last_error()
    bad.grid = 64
    bad.n_obst = 65
    assert lib.ffmp_raster(C.byref(bad), 1, None, None, C.byref(ob), None) == -3
    lidar_cfg = _abi.make_cfg(FFMPConfig(grid=64, n_obst=4, n_beams=8))  # beam_cs NULL
    assert lib.ffmp_reset(C.byref(lidar_cfg), 1, 0, None, 1, C.byref(st), C.byref(ob), None) == -3
    table = (C.c_double * 40)()  # the beam table is read as 16-B {cos, sin} pairs: 8-B aligned is refused
    base = C.cast(table, C.c_void_p).value
    lidar_cfg.beam_cs = base + (8 if base % 16 == 0 else 0)
    assert lib.ffmp_reset(C.byref(lidar_cfg), 1, 0, None, 1, C.byref(st), C.byref(ob), None) == -3
    assert b"16-byte aligned" in lib.ffmp_last_error()
    assert lib.ffmp_scan_collision(-1, 4, None, 0.13, None, None, None) == -1
    # n == 0 with valid pointers is a no-op success (no launch)
    dummy = (C.c_double * 8)()
    p = C.cast(dummy, C.c_void_p).value
    st2 = _abi.StateT(p, p, p, p, p, p, p, p, p)
    ob2 = _abi.ObsT(p, p, p, p, p, p, p)
    out2 = _abi.OutT(p, p, p, p, p)
    assert lib.ffmp_step_state(C.byref(cfg), 0, 0, p, C.byref(st2), C.byref(ob2), C.byref(out2), None) == 0
    assert lib.ffmp_raster(C.byref(cfg), 0, p, None, C.byref(ob2), None) == 0
    # the skewed step (raster of step t + env step of step t + 1): the env step must write the other
    # record buffer; float32 frames without flow planes only; n == 0 launches nothing
    other = C.cast((C.c_double * 8)(), C.c_void_p).value
    assert lib.ffmp_step_skewed(C.byref(cfg), 0, 0, p, C.byref(st2), C.byref(ob2), C.byref(out2), other, 0, 0,
                                None) == 0
    assert lib.ffmp_step_skewed(C.byref(cfg), 4, 0, p, C.byref(st2), C.byref(ob2), C.byref(out2), p, 0, 0,
                                None) == -1
    assert b"other record buffer" in lib.ffmp_last_error()
    assert lib.ffmp_step_skewed(C.byref(cfg), 4, 0, None, C.byref(st2), C.byref(ob2), C.byref(out2), other, 0, 0,
                                None) == -1
    ob2.format = _abi.OBS_U8F16
    assert lib.ffmp_step_skewed(C.byref(cfg), 4, 0, p, C.byref(st2), C.byref(ob2), C.byref(out2), other, 0, 0,
                                None) == -1
    assert b"float32 frames" in lib.ffmp_last_error()
    ob2.format = _abi.OBS_F32
    # observation formats (FFMP_OBS_*): unknown ones are refused; the compact one takes binary16 flow planes
    ob2.format = 7
    assert lib.ffmp_raster(C.byref(cfg), 0, p, None, C.byref(ob2), None) == -1
    assert b"obs.format" in lib.ffmp_last_error()
    assert lib.ffmp_step_fused(C.byref(cfg), 0, 0, p, C.byref(st2), C.byref(ob2), C.byref(out2), 0, None) == -1
    ob2.format = _abi.OBS_U8F16
    assert lib.ffmp_raster(C.byref(cfg), 0, p, None, C.byref(ob2), None) == 0
    flow_cfg = _abi.make_cfg(FFMPConfig(grid=64, n_obst=4, n_beams=0, flow=True))
    ob2.flow = p
    assert lib.ffmp_raster(C.byref(flow_cfg), 0, p, None, C.byref(ob2), None) == 0


def test_header_constants_match_the_binding():
    import re
    h = open(_abi.HEADER_PATH).read()
    assert int(re.search(r"#define FFMP_PACKED_ARG_BEAMS (\d+)", h).group(1)) == _abi.PACKED_ARG_BEAMS
    assert int(re.search(r"#define FFMP_ABI_VERSION (\d+)", h).group(1)) == _abi.ABI_VERSION


def test_config_validation():
    with pytest.raises(ValueError):
        FFMPConfig(grid=66)
    with pytest.raises(ValueError):
        FFMPConfig(n_obst=65)
    with pytest.raises(ValueError):
        FFMPConfig(n_beams=2000)
    c = FFMPConfig(grid=256, n_beams=0)
    assert c.mode == 1 and FFMPConfig(grid=256).mode == 3
    assert c.W == 256 * 0.05 and c.lidar_range == 128 * 0.05


def test_f32_constants_exact():
    c = preset("C3")
    f = c.f32_constants()
    assert f["half_f"] == np.float32(0.5 * (256 * 0.05))
    # cell G/2 is the robot centre exactly (ego coordinate 0)
    assert np.float32(128) * f["res_f"] - f["half_f"] == 0.0
    for G in (64, 100, 128, 256, 512):
        ff = FFMPConfig(grid=G).f32_constants()
        assert np.float32(G // 2) * ff["res_f"] - ff["half_f"] == 0.0, G
    cc = _abi.make_cfg(c)
    for k, v in f.items():
        assert np.float32(getattr(cc, k)) == v


def test_presets_match_baseline():
    import json
    with open(os.path.join(os.path.dirname(HEADER), "..", "BASELINE.json")) as fh:
        cfgs = json.load(fh)["configs"]
    assert len(cfgs) == 5
    for name, txt in zip(("C1", "C2", "C3", "C4", "C5"), cfgs):
        p = PRESETS[name]
        c = preset(name)
        assert f"{c.grid}×{c.grid}" in txt
        assert f"{c.n_obst} " in txt
        if name != "C1":
            assert f"{p['n_envs']}" in txt.replace(",", "")
        if c.n_beams and name != "C4":
            assert f"{c.n_beams}-beam" in txt


def test_beam_table():
    t = beam_table(180)
    assert t.shape == (180, 2)
    assert t[0, 0] == math.cos(-math.pi) and t[0, 1] == math.sin(-math.pi)
    assert np.allclose(np.hypot(t[:, 0], t[:, 1]), 1.0)


def test_bytes_model():
    b = bytes_per_env_step(preset("C3"))
    assert b["raster"] == 12 * 256 * 256 + 4 * (16 + 12 * 16)
    assert bytes_per_env_step(preset("C3", flow=True))["raster"] == 20 * 256 * 256 + 4 * (16 + 12 * 16)
    # frame window W: the older frame is written on 1 step in W-1 (plus resets, counted by bench.py)
    assert bytes_per_env_step(preset("C3"), window=8)["raster"] == 8 * 65536 + (4 * 65536) // 7 + 4 * (16 + 12 * 16)
    assert bytes_per_env_step(preset("C3"), window=2)["raster"] == b["raster"]
    # seamless ring: never wraps, only the new frame (plus resets)
    assert bytes_per_env_step(preset("C3"), window=8, seamless=True)["raster"] == 8 * 65536 + 4 * (16 + 12 * 16)
    assert bytes_per_env_step(preset("C3"), window=2, seamless=True)["raster"] == b["raster"]
    assert b["total"] > b["raster"]
    # compact format: 1-byte frames, 2-byte potential
    assert bytes_per_env_step(preset("C3"), window=8, seamless=True, obs_format="u8f16")["raster"] == \
        3 * 65536 + 4 * (16 + 12 * 16)
    assert bytes_per_env_step(preset("C3"), obs_format="u8f16")["raster"] == 4 * 65536 + 4 * (16 + 12 * 16)


def test_bench_traffic_lookup():
    """bench.py reads roofline.traffic from the committed PMC summary of the same configuration
    (step kind, frame window, ring, obs format), else reports null."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(os.path.dirname(HEADER), "..", "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    prof = os.path.join(os.path.dirname(HEADER), "..", "profiles")
    for name, fused, fmt in (("C3", False, "f32"), ("C3", True, "f32"), ("C3", False, "u8f16"), ("C3", True, "u8f16")):
        label = name + ("" if fmt == "f32" else "_" + fmt) + ("_fused" if fused else "")
        path = os.path.join(prof, f"pmc_traffic_{label}.json")
        if not os.path.exists(path):
            continue
        d = json.load(open(path))
        got, src = bench.load_traffic(name, d["n_envs"], d["frame_window"], d["ring"], fused, fmt)
        assert got == d["raster_hbm_bytes_per_launch"]
        # the line names the profile the figure came from (roofline.traffic_source)
        assert os.path.samefile(os.path.join(prof, "..", src), path)
        assert bench.load_traffic(name, d["n_envs"] + 1, d["frame_window"], d["ring"], fused, fmt) == (None, None)
        assert bench.load_traffic(name, d["n_envs"], d["frame_window"] + 1, d["ring"], fused, fmt) == (None, None)
    assert bench.load_traffic("C3", 32768, 8, "seamless", False, "u8f16") != bench.load_traffic("C3", 32768, 8,
                                                                                               "seamless", False)


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(_abi.FFMPBackendError):
        _abi.load(str(tmp_path / "nope.so"))


def test_product_never_imports_oracle():
    root = os.path.join(os.path.dirname(HEADER), "..", "flow_field_based_motion_planner_amd")
    for dp, _, files in os.walk(root):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, flags=re.M), f


def test_episode_abi_validation_no_gpu(lib):
    dummy = (C.c_double * 8)()
    p = C.cast(dummy, C.c_void_p).value
    ep = _abi.EpisodeT(*([p] * 9))
    out = _abi.OutT(p, p, p, p, p)
    assert lib.ffmp_episode_update(4, C.byref(out), 0, 0, 0.8, 1, C.byref(ep), None) == -1
    assert b"window" in lib.ffmp_last_error()
    assert lib.ffmp_episode_update(4, C.byref(out), 65, 0, 0.8, 1, C.byref(ep), None) == -1
    assert lib.ffmp_episode_update(4, C.byref(out), 10, -1, 0.8, 1, C.byref(ep), None) == -1
    assert lib.ffmp_episode_update(4, C.byref(_abi.OutT(p, p, None, p, p)), 10, 0, 0.8, 1, C.byref(ep), None) == -1
    bad = _abi.EpisodeT(*([p] * 9))
    bad.step = None
    assert lib.ffmp_episode_init(4, None, 0, C.byref(bad), None) == -1
    assert lib.ffmp_episode_update(0, C.byref(out), 10, 0, 0.8, 1, C.byref(ep), None) == 0
    assert lib.ffmp_episode_init(-1, None, 0, C.byref(ep), None) == -1


def test_dlpack_view_over_host_memory(lib):
    """ffmp_dlpack + the capsule hand-off (how the seamless ring reaches torch), exercised on
    host memory: shape, element strides (incl. a padded slot stride), aliasing, lifetime."""
    import gc

    import torch

    from flow_field_based_motion_planner_amd import _abi
    a = np.arange(3 * 20, dtype=np.float32)
    t = _abi.tensor_from_pointer(a.ctypes.data, (3, 2, 4), (20, 4, 1), _abi.DL_CPU, 0)
    assert t.shape == (3, 2, 4) and t.stride() == (20, 4, 1) and t.dtype == torch.float32
    assert float(t[2, 1, 3]) == a[2 * 20 + 1 * 4 + 3]
    v = t[1:3].transpose(0, 1)  # the state_m-style pair view
    del t
    gc.collect()
    a[20] = -5.0  # a view, not a copy
    assert float(v[0, 0, 0]) == -5.0
    assert not lib.ffmp_dlpack(None, 1, 0, 1, None, None, 32, None)  # bad arguments -> NULL


def test_ring_api_without_gpu(lib):
    """The ring helper validates its arguments and, without a GPU, fails with a message."""
    import ctypes as C
    ring, base, stride = C.c_void_p(), C.c_void_p(), C.c_int64()
    assert lib.ffmp_ring_create(0, 0, 4, None, 0, C.byref(ring), C.byref(base), C.byref(stride)) == -1
    assert lib.ffmp_ring_create(0, 4096, 1, None, 0, C.byref(ring), C.byref(base), C.byref(stride)) == -1
    assert lib.ffmp_ring_create(0, 4096, 4, C.c_void_p(16), 0, C.byref(ring), C.byref(base), C.byref(stride)) == -1
    rc = lib.ffmp_ring_create(0, 1 << 20, 4, None, 0, C.byref(ring), C.byref(base), C.byref(stride))
    assert rc == -2 and not ring.value and b"ffmp_ring" in lib.ffmp_last_error()
    assert lib.ffmp_ring_rebuild(None, 1, None, 0, C.byref(ring), C.byref(base), C.byref(stride)) == -1
    assert lib.ffmp_ring_destroy(None) == 0
    assert lib.ffmp_ring_pool_bytes(-1) == 0
    info = (C.c_double * 5)()
    assert lib.ffmp_ring_info(None, info, 5) == -1
    # FFMP_TUNE_RING_EXTRA: 0 = default, v = at most v - 1 extra pairing pieces; negative refused
    assert lib.ffmp_set_tuning(_abi.TUNE_RING_EXTRA, -1) == -1
    prev = lib.ffmp_set_tuning(_abi.TUNE_RING_EXTRA, 5)
    assert prev == 0 and lib.ffmp_set_tuning(_abi.TUNE_RING_EXTRA, prev) == 5


def test_exact_math_domain_validation_no_gpu(lib):
    """The raster's sqrt_rn / rcp_rn are exact on rho_min in [2^-48, 2^100], obst_rmin >= 0
    (ffmp_device.h); check_cfg refuses configurations outside that domain before any launch."""
    ob = _abi.ObsT()
    for field, val in (("rho_min_f", 0.0), ("rho_min_f", 2.0 ** -60), ("rho0_f", float("inf")),
                       ("rho_min_f", float("nan")), ("obst_rmin", -0.1)):
        bad = _abi.make_cfg(FFMPConfig(grid=64, n_obst=4, n_beams=0))
        setattr(bad, field, val)
        assert lib.ffmp_raster(C.byref(bad), 1, None, None, C.byref(ob), None) == -3, field
    assert b"rho" in lib.ffmp_last_error() or b"obst_rmin" in lib.ffmp_last_error()
    assert lib.ffmp_check_exact_math(2, 0, 1, None, None, None) == -1
    assert lib.ffmp_check_exact_math(0, 0, 1, None, None, None) == -1
