"""The C ABI used from plain C (tests/c_abi_consumer.c): no Python, no torch in the consumer.

CPU: the consumer compiles with gcc against include/ffmp.h and links libffmp.so.
GPU: it runs on cuda:0 — reset + 25 steps of 512 envs with moving discs and lidar — and checks
size-independent invariants (frame hand-over, reset frames, gradient vs potential plane,
is_collision2 on the lidar output).  This is the integration a C/C++ host (or a cgo / JNI
binding) would do against the shared library."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "flow_field_based_motion_planner_amd", "lib")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _build(lib, out):
    assert lib is not None  # fixture builds libffmp.so
    cmd = ["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROCM, "include"),
           os.path.join(ROOT, "tests", "c_abi_consumer.c"), "-o", out,
           "-L", LIBDIR, "-lffmp", "-L", os.path.join(ROCM, "lib"), "-lamdhip64",
           f"-Wl,-rpath,{LIBDIR}", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}", "-lm"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return out


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not on PATH")
def test_c_consumer_compiles(lib, tmp_path):
    _build(lib, str(tmp_path / "c_abi_consumer"))


@pytest.mark.gpu
def test_c_consumer_runs(lib, tmp_path):
    exe = _build(lib, str(tmp_path / "c_abi_consumer"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout}\n{r.stderr}"
    assert "c_abi_consumer ok" in r.stdout
