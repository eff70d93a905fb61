"""The §5 sanitizer leg: the CPU oracle built with AddressSanitizer + UndefinedBehaviorSanitizer
(oracle/sanitize_main.c) runs C2/C3/C4 at full player/NPC counts through reset, scripted and
random actions, culls and auto-resets, a forced episode end, a state round trip and the event
log. A report of either sanitizer fails the run (-fno-sanitize-recover=all)."""

import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "sanitize"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ORACLE, "build", "oracle_sanitize"), "90"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    for name in ("C2", "C3", "C4"):
        assert f"{name}: 90 ticks" in r.stdout
