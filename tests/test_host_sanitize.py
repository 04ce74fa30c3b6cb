"""Sanitizers on the host code of the C ABI (SURVEY §5 "race detection / sanitizers": the path
has no host threads, so what is left to check is the host side of libffmp — validation,
footprint, layout / tuning queries, the DLPack wrapper and its deleter, the ring pool).

libffmp is rebuilt with AddressSanitizer + UndefinedBehaviorSanitizer on its HOST code only
(`-Xarch_host -fsanitize=...`; GPU code is never sanitized here) and driven by the plain-C
program tests/abi_sanitize.c through every entry point that needs no GPU.  LeakSanitizer runs
too.  CPU only (~40 s, most of it the device-code compile that the shared library still needs).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CLANG = "/opt/rocm/llvm/bin/clang"
SRCS = [os.path.join(ROOT, "flow_field_based_motion_planner_amd", "csrc", f) for f in ("ffmp_kernels.hip", "ffmp_ring.hip")]


@pytest.mark.skipif(not (shutil.which(HIPCC) and os.path.exists(CLANG)), reason="ROCm toolchain absent")
def test_abi_host_code_under_asan_ubsan(tmp_path):
    lib = tmp_path / "libffmp_san.so"
    san = ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined"]
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-ffp-contract=off", "-fPIC",
                    "-shared", "-I" + os.path.join(ROOT, "include")] + san + ["-o", str(lib)] + SRCS,
                   check=True, capture_output=True, cwd=str(tmp_path))
    exe = tmp_path / "abi_sanitize"
    # -fno-sanitize=function: the C program declares its own DLManagedTensor type (as any DLPack
    # consumer does), which the indirect-call type check would flag against the C++ one
    subprocess.run([CLANG, "-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize=function",
                    "-fno-sanitize-recover=undefined", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "abi_sanitize.c"), "-L" + str(tmp_path), "-lffmp_san",
                    "-Wl,-rpath," + str(tmp_path), "-o", str(exe)], check=True, capture_output=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=120)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report
    assert "all host-side checks passed" in r.stdout
    assert "AddressSanitizer" not in report and "runtime error" not in report and "LeakSanitizer" not in report
