"""conv2's forward (32 -> 64, k = 32, 69^2 -> 38^2) at B = 256: 768 workgroups of 512 positions for
512 resident slots (2 per CU) leave the second round half empty.  Times one launch, three launches
in sequence and three on three streams at once (the replay's Q(s), Q_main(s') and Q_target(s')
are independent).  FFMP_CONV_MBW=1/2/4 forces the tile (read once per process)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.conv_mfma import conv2d_nhwc, pack_weight  # noqa: E402

dev = torch.device("cuda:0")
B = 256
flop = 2.0 * B * 38 * 38 * 64 * 32 * 32 * 32
xs = [torch.relu(torch.randn(B, 69, 69, 32, device=dev)).to(torch.bfloat16) for _ in range(3)]
w = pack_weight((torch.randn(64, 32, 32, 32, device=dev) / 181.0))
bias = torch.randn(64, device=dev)
streams = [torch.cuda.Stream(dev) for _ in range(3)]


def one(i=0):
    return conv2d_nhwc(xs[i], w, bias, relu=True, out_dtype=torch.bfloat16)


def seq():
    for i in range(3):
        one(i)


def par():
    cur = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    ev.record(cur)
    for i, s in enumerate(streams):
        s.wait_event(ev)
        with torch.cuda.stream(s):
            one(i)
    for s in streams:
        cur.wait_stream(s)


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


tag = os.environ.get("FFMP_CONV_MBW", "auto")
for rep in range(2):
    t1, t3, tp = timeit(one), timeit(seq), timeit(par)
    print(f"MBW {tag}: one {t1:.3f} ms ({flop / t1 / 1e9:.0f} TFLOP/s)  three in sequence {t3:.3f} ms  "
          f"three on three streams {tp:.3f} ms ({3 * flop / tp / 1e9:.0f} TFLOP/s)", flush=True)
