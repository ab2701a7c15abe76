#!/bin/bash
# Round 5, HEAD with 4,096 hot words in LDS: the whole GPU suite, the suite with labels forced, the
# measurement-variant tests, smoke, then rocprofv3 summaries of configs[1] and configs[2].
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13a; mkdir -p $out
T="timeout -k 10"
cd $R
$T 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $out/gpu_tests.log 2>&1
rc=$?; tail -3 $out/gpu_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "gpu tests rc=$rc"; exit 1; }
FGI_LABELS=1 $T 400 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $out/gpu_tests_labels.log 2>&1
rc=$?; tail -3 $out/gpu_tests_labels.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "forced-label gpu tests rc=$rc"; exit 1; }
FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_variants.so $T 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_probe_summary.py -q --timeout 200 --timeout-method thread > $out/variants_tests.log 2>&1
rc=$?; tail -2 $out/variants_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "variant tests rc=$rc"; exit 1; }
$T 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke rc=$?"; tail -20 $out/smoke.log; exit 1; }
tail -1 $out/smoke.log
bash profiles/run_profile.sh r13c1 --config rmat24 --no-secondary --no-cpu --no-e2e --steps 10 --warmup 2 > $out/prof_c1.log 2>&1 || { echo "profile c1 rc=$?"; tail -20 $out/prof_c1.log; exit 1; }
bash profiles/run_profile.sh r13c2 --config rmat27 --no-secondary --no-cpu --no-e2e --steps 10 --warmup 2 > $out/prof_c2.log 2>&1 || { echo "profile c2 rc=$?"; tail -20 $out/prof_c2.log; exit 1; }
echo "profiles done"
