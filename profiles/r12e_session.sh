#!/bin/bash
# Round 5: BASELINE.json's other configurations on HEAD (bench_configs.py: configs[4] streaming rounds,
# configs[3] churn + prune, configs[0] with the CPU oracle), and the measurement-variant tests
# (FGI_LIBRARY = libfgi_variants.so: fused waves, probe summary).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12e; mkdir -p $out
T="timeout -k 10"
cd $R
$T 600 python bench_configs.py > $out/configs.jsonl 2> $out/configs.err || { echo "configs rc=$?"; tail -20 $out/configs.err; exit 1; }
cut -c1-600 $out/configs.jsonl
FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_variants.so $T 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_probe_summary.py -q --timeout 200 --timeout-method thread > $out/variants_tests.log 2>&1
rc=$?; tail -4 $out/variants_tests.log
