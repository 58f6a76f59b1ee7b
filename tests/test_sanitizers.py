"""Host-native code under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5 race
detection / sanitizers): tools/sanitize_runtime.py builds the C++ serving runtime (BlockPool,
BPE, pack_decode, the shared-memory StepChannel) with -fsanitize=address,undefined and runs a
threaded stress of every entry point in a child interpreter; any sanitizer report fails the test.
(GPU-side ASan / XNACK builds are not available on this pool; the HIP kernels are covered by the
fp32-reference numerics tests instead.)"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_runtime_clean_under_asan_ubsan():
    if shutil.which("g++") is None:
        pytest.skip("no host C++ compiler")
    lib = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    if not os.path.isabs(lib) or not os.path.exists(lib):
        pytest.skip("no ASan runtime")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sanitize_runtime.py")], capture_output=True,
                       text=True, timeout=900, cwd=ROOT)
    assert r.returncode == 0 and "clean" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
