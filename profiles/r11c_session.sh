#!/bin/bash
# Round 5: the labelled `_usedBy` diagnostic, then the new tests (labels, async waves, host-collective
# partitions) without stopping at the first failure, then the whole GPU suite and the whole suite with
# labels forced on every graph.
set -u
out=gpurun_out/r11c; mkdir -p $out
T="timeout -k 10"
$T 240 python -u profiles/r11c_usedby_diag.py > $out/diag.log 2>&1 || { echo "diag rc=$?"; tail -30 $out/diag.log; exit 1; }
cat $out/diag.log
$T 400 python -u -m pytest tests/test_gpu_labels.py tests/test_gpu_async.py tests/test_gpu_part_host.py tests/test_gpu_part_plan.py -v --timeout 120 --timeout-method thread > $out/new_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $out/new_tests.log | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "new tests rc=$rc"; exit 1; }
DES="--deselect tests/test_gpu_labels.py::test_labelled_mutations_batches_and_prune"
$T 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread $DES > $out/gpu_tests.log 2>&1
rc=$?; tail -15 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests rc=$rc"; exit 1; }
FGI_LABELS=1 $T 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread $DES > $out/gpu_tests_labels.log 2>&1
rc=$?; tail -15 $out/gpu_tests_labels.log
