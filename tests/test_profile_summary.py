"""tools/summarize_profiles.py's dispatch bookkeeping of bench.py's timed graph replays (host only): the
dispatches per full replay and per remainder replay for the two-launch, one-launch and skewed graphs, and
the per-replay HBM bytes it sums from a synthetic PMC file."""
import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_spec = importlib.util.spec_from_file_location("summarize_profiles", os.path.join(ROOT, "tools", "summarize_profiles.py"))
sp = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(sp)


def _bj(fused=False, skewed=False, rem=0, replays=3, gs=8):
    return {"config": {"fused": fused, "graph": {"steps_per_replay": gs, "replays": replays, "remainder_steps": rem,
                                                 "skewed": skewed}}}


def test_replay_dispatches():
    assert sp.replay_dispatches(_bj(), 8) == (16, 0)
    assert sp.replay_dispatches(_bj(rem=4), 8) == (16, 8)
    assert sp.replay_dispatches(_bj(fused=True, rem=4), 8) == (8, 4)
    # skewed: env(0) + 7 skewed launches + raster(7); an even remainder is skewed too, an odd one two-launch
    assert sp.replay_dispatches(_bj(skewed=True), 8) == (9, 0)
    assert sp.replay_dispatches(_bj(skewed=True, rem=4), 8) == (9, 5)
    assert sp.replay_dispatches(_bj(skewed=True, rem=3), 8) == (9, 6)


def test_step_kernels_orders_and_filters(tmp_path):
    path = tmp_path / "run_counter_collection.csv"
    rows = [(3, "void raster_kernel<true>(...)", 5.0), (1, "void env_kernel<0>(...)", 1.0),
            (2, "void skew_kernel<true, true, 16>(...)", 6.0), (4, "other_kernel", 99.0),
            (5, "void skew_kernel<true, true, 16>(...)", 7.0)]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for d, k, v in rows:
            w.writerow({"Dispatch_Id": d, "Kernel_Name": k, "Counter_Name": "WRITE_SIZE", "Counter_Value": v})
        w.writerow({"Dispatch_Id": 6, "Kernel_Name": "void env_kernel<0>(...)", "Counter_Name": "FETCH_SIZE",
                    "Counter_Value": 3.0})
    got = sp.step_kernels(str(path), "WRITE_SIZE")
    assert got == [("env_kernel", 1.0), ("skew_kernel", 6.0), ("raster_kernel", 5.0), ("skew_kernel", 7.0)]
    per = sp.counters(str(path), "WRITE_SIZE")
    assert per["skew_kernel"] == [6.0, 7.0] and per["raster_kernel"] == [5.0] and per["env_kernel"] == [1.0]
