"""The CPU restatement (oracle/, the checker of every parity test) built with
AddressSanitizer + UndefinedBehaviorSanitizer and driven through every entry
point (oracle/sanitize_driver.cpp): no out-of-bounds access, use after free,
leak, signed overflow, bad shift or misaligned access in the checker."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oracle_clean_under_asan_ubsan():
    odir = os.path.join(ROOT, "oracle")
    subprocess.run(["make", "-s", "-C", odir, "sanitize"], check=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               OMP_NUM_THREADS="2")
    r = subprocess.run([os.path.join(odir, "sanitize_driver")], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize_driver ok" in r.stdout
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr, r.stderr
