#!/bin/bash
# GPU tests of the current build, A/B against the previous build, then the level traces and the
# other configs (first half of the r5b measurements). Usage: bash profiles/r5c_session.sh <tag>
set -u
tag=$1
R=$(pwd)
out=$R/gpurun_out/$tag
mkdir -p "$out"
FGI_PART_MEM_OUT=$out/part_mem.json timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -2 "$out/gpu_tests.log"
if [ $rc -ne 0 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
bash profiles/r5_ab.sh ${tag}_ab 3 stl.fusion_amd/lib/libfgi_base.so stl.fusion_amd/lib/libfgi.so || exit 1
for cfg in rmat24 rmat27 layered_1m; do
  FGI_TRACE=1 timeout -k 10 180 python profiles/wave_levels.py $cfg > "$out/levels_$cfg.out" 2> "$out/levels_$cfg.err" || { echo "levels $cfg rc=$?"; exit 1; }
done
echo "levels done"
timeout -k 10 300 python bench_configs.py --no-cpu > "$out/configs.jsonl" 2> "$out/configs.err" || { echo "configs rc=$?"; exit 1; }
echo "configs done"
