"""Host-side sanitizer runs of lumen's C++ code (no GPU): the CPU AdamW used by ZeRO-Offload is
built with AddressSanitizer + UndefinedBehaviorSanitizer into a small harness and checked against
a double-precision reference at sizes around the 16-wide vector and 64 Ki-element chunk edges,
once on the AVX-512 path (when the host has it) and once on the portable path."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "lumen", "csrc", "cpu", "cpu_adam.cpp")
HARNESS = os.path.join(ROOT, "tests", "native", "cpu_adam_harness.cpp")


@pytest.mark.parametrize("portable", [False, True])
def test_cpu_adam_asan_ubsan(tmp_path, portable):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path / "cpu_adam_asan")
    cmd = [cxx, "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=undefined", "-fopenmp", "-std=c++17", SRC, HARNESS, "-o", exe]
    if portable:
        cmd.insert(1, "-DLUMEN_NO_AVX512")
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0",
               OMP_NUM_THREADS="4")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout + r.stderr)[-3000:]
