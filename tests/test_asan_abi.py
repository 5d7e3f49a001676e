"""the C-ABI's host code under AddressSanitizer in the CPU-only build (no GPU).

tools/asan_abi.py compiles every csrc/*.hip with the host side instrumented
(-Xarch_host -fsanitize=address) into libregcn_hip_asan.so and links a harness generated from
include/regcn_hip.h against it.  Every int-returning export is called with NULL pointers, the
descriptor-taking ones with all-zero descriptors, exports with a row width with d = -4 (and
d = 1000 where only d <= 256 is built), the Givens rotation with misaligned pairs (the ABI's
view of an odd width) and a negative pair count, the builders with a 1-byte workspace and the
cross entropy with none: each must return a negative REGCN_E* code before any HIP call (with
no GPU a HIP call would return a positive hipError_t), with no ASan report."""
import os
import shutil
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_capi_validation_under_asan():
    import torch
    if torch.cuda.is_available():
        pytest.skip("CPU-only check: run without a GPU (a missed validation would launch a kernel)")
    if not shutil.which("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "asan_abi.py")], capture_output=True, text=True,
                       timeout=1200)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out
    line = [l for l in r.stdout.splitlines() if l.startswith("asan abi check:")]
    assert line and line[0].endswith(" 0 failed"), out[-2000:]
    n = int(line[0].split()[3])
    assert n >= 120, line  # every export's null case at least
    lib = os.path.join(REPO, "re-gcn_amd", "csrc", "build", "asan", "libregcn_hip_asan.so")
    syms = subprocess.run(["nm", "-D", lib], capture_output=True, text=True).stdout
    assert "__asan_report" in syms  # the host code is instrumented
