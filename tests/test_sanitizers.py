"""Host-side sanitizer runs (SURVEY §5 aux subsystem): the CPU oracle (gcc) and the product's
physics templates instantiated on the host (hipcc, host side only) built with AddressSanitizer +
UndefinedBehaviorSanitizer (tools/san/Makefile, every finding aborts) and driven over random,
saturated and non-finite inputs, leak detection on. GPU-side sanitizers are unavailable on this
pool, so device code is covered by the parity tests instead. The first run (round 3) found
undefined behaviour in the host instantiation of q_sincos (int() of a diverged angle), fixed by
quadrant_of in quad_physics.h."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tools", "san")


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("needs gcc and hipcc")
    subprocess.run(["make", "-s", "-C", SAN], check=True, timeout=600)
    return os.path.join(SAN, "_build")


@pytest.mark.parametrize("prog", ["san_oracle", "san_physhost"])
def test_sanitized_run_is_clean(built, prog):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(built, prog)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and f"{prog} OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
