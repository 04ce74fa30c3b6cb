"""Can the env step of step i + 1 run beside the raster of step i on a few CUs of its own?  C3 steps timed
(HIP events on the raster's stream) as: the two-launch step graph (serial), and live two-stream steps
(the pipelined schedule: env kernels on a side stream with two record buffers, rasters on the main
stream) whose side stream is unmasked or restricted to n CUs (hipExtStreamCreateWithCUMask).
usage: python tools/masked_env_probe.py [preset] [n_envs]"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 32768
dev = torch.device("cuda:0")
hip = C.CDLL("libamdhip64.so")


def masked_stream(n_cu: int):
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    words = [0] * ((ncu + 31) // 32)
    per_xcd = ncu // 8
    for j in range(n_cu):  # spread over the 8 XCDs
        cu = (j % 8) * per_xcd + j // 8
        words[cu // 32] |= 1 << (cu % 32)
    arr = (C.c_uint32 * len(words))(*words)
    s = C.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(C.byref(s), len(words), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


env = FFMPVec(n, name, device=dev, fused=False)
env.reset()
acts = torch.randint(0, 28, (8, n), device=dev)
for i in range(16):
    env.step(acts[i % 8])
torch.cuda.synchronize()
k = env.graph_period()
main = torch.cuda.current_stream(dev)


def live_pipelined(side, reps):
    rec0 = env.record
    if getattr(env, "_record_alt", None) is None:
        env._record_alt = torch.empty_like(rec0)
    bufs = (rec0, env._record_alt)
    ev_ras_prev = [None, None]
    for _ in range(reps):
        fork = torch.cuda.Event()
        fork.record(main)
        side.wait_event(fork)
        ev_ras = []
        for i in range(k):
            buf = bufs[(i + 1) % 2]
            env.record = buf
            env._state_c.record = buf.data_ptr()
            with torch.cuda.stream(side):
                if i >= 2:
                    side.wait_event(ev_ras[i - 2])
                env.step_state(acts[i])
                ee = torch.cuda.Event()
                ee.record(side)
            main.wait_event(ee)
            env.raster_step()
            er = torch.cuda.Event()
            er.record(main)
            ev_ras.append(er)
        env.record = rec0
        env._state_c.record = rec0.data_ptr()
    return ev_ras_prev


def timed(fn, reps=12):
    fn(2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    fn(reps)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (reps * k)


g = env.capture(k, skewed=False)


def serial(reps):
    for _ in range(reps):
        g.replay(acts[:k])


variants = [("serial graph", serial), ("live, side unmasked", lambda r: live_pipelined(torch.cuda.Stream(dev), r))]
for ncu in (8, 16, 32, 64):
    s = masked_stream(ncu)
    variants.append((f"live, side on {ncu} CUs", (lambda s_: (lambda r: live_pipelined(s_, r)))(s)))
for rnd in range(2):
    for nm, fn in variants:
        ms = timed(fn)
        print(f"{name} n={n} round {rnd} {nm:24s}: {ms * 1e3:8.1f} us/step  {n / ms / 1e3:7.2f} M env-steps/s", flush=True)
env.check_errors()
