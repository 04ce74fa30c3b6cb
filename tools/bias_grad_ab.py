"""The conv layers' bias gradients (sum of the bf16 output gradient over batch and positions, fp32
accumulation) at B = 256: torch's one-shot g.sum((0, 1, 2)) against a two-stage per-sample sum.
usage: python tools/bias_grad_ab.py"""
import torch

dev = torch.device("cuda:0")


def timeit(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for H, N in ((69, 32), (38, 64), (31, 64), (24, 64), (17, 64), (10, 64)):
    g = torch.randn(256, H, H, N, device=dev).to(torch.bfloat16)
    a = lambda: g.sum((0, 1, 2), dtype=torch.float32)  # noqa: E731
    b = lambda: g.sum((1, 2), dtype=torch.float32).sum(0)  # noqa: E731
    c = lambda: g.view(256 * H, H * N).sum(0, dtype=torch.float32).view(H, N).sum(0)  # noqa: E731
    ref = g.double().sum((0, 1, 2))
    errs = [float((f().double() - ref).abs().max()) for f in (a, b, c)]
    print(f"{H}^2 x {N}: one-shot {timeit(a):6.1f} us  per-sample {timeit(b):6.1f} us  row-sum {timeit(c):6.1f} us  "
          f"max err {errs[0]:.2e} {errs[1]:.2e} {errs[2]:.2e}", flush=True)
