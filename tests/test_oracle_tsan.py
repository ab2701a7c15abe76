"""The oracle's threaded paths under ThreadSanitizer (CPU only).

oracle/Makefile's `tsan` target builds oracle/tsan_roots.cpp with -fsanitize=thread: the
parallel-over-roots cascade (bench.py's cpu_baseline leg) at 2/4/8 threads must reproduce the
sequential result exactly, and TSAN must report no data race in it or in the threaded bulk
operations (R-MAT generator, tags, import, snapshot/restore). A TSAN report exits with 66.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(ROOT, "oracle")


def test_parallel_over_roots_under_tsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "tsan"], check=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([os.path.join(ORACLE, "build", "tsan_roots"), "14"], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ThreadSanitizer" not in r.stderr
    assert r.stdout.count(" same") == 3 and r.stdout.rstrip().endswith("ok")
