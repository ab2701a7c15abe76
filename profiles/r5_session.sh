#!/bin/bash
# Round-3 GPU session: GPU tests, then bench.py (only if the tests ended normally: exit 0 / 1).
# usage: bash profiles/r5_session.sh <tag> [pytest selector...]
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
sel=${*:-tests}
FGI_PART_MEM_OUT=$out/part_mem.json FGI_FANOUT_OUT=$out/fanout.json timeout -k 10 900 python -u -m pytest $sel -m gpu -v --timeout 300 --timeout-method thread > "$out/gpu_tests.log" 2>&1
rc=$?
tail -3 "$out/gpu_tests.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: no further GPU step"; exit $rc; fi
timeout -k 10 300 python bench.py > "$out/bench.json" 2> "$out/bench.err"
rc2=$?
echo "bench rc=$rc2"
exit $rc2
