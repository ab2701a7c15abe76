#!/bin/bash
# Head bitmaps for pull probes. libfgi: cold heads (heads that are not hot) probe a head-only bitmap past
# the hot snapshot, plus small-pull-level trims (hot staging skipped below 1,024 candidates, only changed
# visit words written back). libfgi_headfreq: every head ranked by count, its bit kept where its
# invalidated bit is (no snapshot gather). GPU tests, the probe-mix microbenchmark, then an A/B against
# HEAD's build (libfgi_base) on configs[1] and configs[2]'s graph.
set -u
out=gpurun_out/r6b
mkdir -p "$out"
L=stl.fusion_amd/lib
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$out/gpu_tests.log" 2>&1 \
    || { echo "tests rc=$?"; tail -30 "$out/gpu_tests.log"; exit 1; }
tail -2 "$out/gpu_tests.log"
FGI_LIBRARY=$PWD/$L/libfgi_headfreq.so timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_scenarios.py tests/test_gpu_golden.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests_headfreq.log" 2>&1 \
    || { echo "tests headfreq rc=$?"; tail -30 "$out/tests_headfreq.log"; exit 1; }
tail -1 "$out/tests_headfreq.log"
FGI_LIBRARY=$PWD/$L/libfgi_h1eager.so timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > "$out/tests_h1eager.log" 2>&1 \
    || { echo "tests h1eager rc=$?"; tail -30 "$out/tests_h1eager.log"; exit 1; }
tail -1 "$out/tests_h1eager.log"
bash profiles/r5_ab.sh r6b_ab24 3 $L/libfgi_base.so $L/libfgi_h1eager.so $L/libfgi.so $L/libfgi_headfreq.so || exit 1
bash profiles/r5_ab.sh r6b_ab27 1 --args --config rmat27 -- $L/libfgi_base.so $L/libfgi_h1eager.so $L/libfgi.so $L/libfgi_headfreq.so || exit 1
