"""AddressSanitizer + UndefinedBehaviorSanitizer over the CPU code (SURVEY.md
5): the oracle's literal restatements, the CPU model of the kernel
arithmetic, the pyramid and legacy restatements, and the host side of the C
ABI (gqmap_host.cpp), driven by tests/native/san_driver.cpp on small inputs
of every engine.  Any sanitizer report aborts the driver (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="needs gcc/g++")
def test_asan_ubsan_cpu_code_clean():
    subprocess.run(["make", "-s", "-C", HERE], check=True, capture_output=True, text=True, timeout=600)
    # verify_asan_link_order=0: the environment may preload a library of its own
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1", OMP_NUM_THREADS="3")
    r = subprocess.run([os.path.join(HERE, "_build", "san_driver")], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "sanitizer driver: clean" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
