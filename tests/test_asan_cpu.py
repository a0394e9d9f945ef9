"""Host AddressSanitizer + UBSan run of the C-ABI's host code (race detection / sanitizers row).

tests/asan/Makefile compiles the product sources with the sanitizers on the host pass only (GPU sanitizers are
not available on this pool) and links tests/asan/abi_asan.cpp, which drives every argument-validation path of
the device entry points, the kernel-selection knobs and cram_passage_weights (random monotone / non-monotone
offset maps, empty prompts, error paths) against a naive restatement of re_weighting.py:105-110.
No GPU is touched.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_abi_host_code_is_asan_and_ubsan_clean():
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("hipcc / make not available")
    d = os.path.join(REPO, "tests", "asan")
    subprocess.run(["make", "-C", d, "-s"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(d, "build", "abi_asan")], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all expectations held" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr
