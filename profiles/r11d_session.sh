#!/bin/bash
# Round 5: the labelled pull diagnostic, then the tests that failed in r11c.
set -u
out=gpurun_out/r11d; mkdir -p $out
T="timeout -k 10"
FGI_TRACE=1 $T 120 python -u profiles/r11d_pull_diag.py > $out/pull_diag.log 2>&1 || { echo "diag rc=$?"; tail -30 $out/pull_diag.log; exit 1; }
grep -E "candidates|labels|lbl|hot" $out/pull_diag.log | head -60
$T 500 python -u -m pytest tests/test_gpu_labels.py tests/test_gpu_async.py tests/test_gpu_part_host.py "tests/test_gpu_parity.py::test_cycles_and_self_loops" tests/test_gpu_configs.py::test_configs2_rmat27_single_gpu_wave -v --timeout 200 --timeout-method thread > $out/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $out/tests.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "tests rc=$rc"; exit 1; }
FGI_LABELS=1 $T 300 python -u -m pytest tests/test_gpu_scale.py::test_pull_grid_geometry_invariance "tests/test_gpu_parity.py::test_cycles_and_self_loops" -v --timeout 200 --timeout-method thread > $out/tests_labels.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $out/tests_labels.log | tail -20
