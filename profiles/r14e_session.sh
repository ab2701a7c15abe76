#!/bin/bash
# Round 6: partition codes (hub-first numbering within each rank's range). GPU suite; the partition suites
# with codes forced on every graph (FGI_LABELS=1); configs[2] in 8 in-process ranks with codes (auto at
# 2^27) against none (FGI_LABELS=-1): wave time, and level-1 FETCH / L2 per rank (one PMC pass each)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14e; mkdir -p $out
T="timeout -k 10"
cd $R
$T 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests.log 2>&1 || { echo "gpu tests rc=$?"; tail -40 $out/gpu_tests.log; exit 1; }
tail -1 $out/gpu_tests.log
FGI_LABELS=1 $T 900 python -u -m pytest tests/test_gpu_part.py tests/test_gpu_part_plan.py tests/test_gpu_part_load.py \
    tests/test_gpu_part_mutations.py tests/test_gpu_part_rccl.py tests/test_gpu_part_host.py tests/test_gpu_bench_multi.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > $out/gpu_tests_codes.log 2>&1 || { echo "codes tests rc=$?"; tail -40 $out/gpu_tests_codes.log; exit 1; }
tail -1 $out/gpu_tests_codes.log
for r in 1 2; do
  $T 300 python profiles/part_local_timing.py 27 8 5 8 >> $out/ab.txt 2>> $out/ab.err || { echo "timing rc=$?"; tail -5 $out/ab.err; exit 1; }
  FGI_LABELS=-1 $T 300 python profiles/part_local_timing.py 27 8 5 8 >> $out/ab.txt 2>> $out/ab.err || { echo "timing rc=$?"; tail -5 $out/ab.err; exit 1; }
done
cat $out/ab.txt
cd /tmp && export TMPDIR=/tmp
for lab in auto -1; do
  for pmc in FETCH_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    name=$(echo "$pmc" | tr ' ' '_')
    env FGI_LABELS=$([ $lab = auto ] && echo 0 || echo -1) timeout -s KILL 240 rocprofv3 --pmc $pmc -T -d $out/pmc_${lab}_$name -o run --output-format csv -- \
        python3 $R/profiles/part_local_timing.py 27 8 1 8 > $out/pmc_${lab}_$name.out 2> $out/pmc_${lab}_$name.err || { echo "pmc rc=$?"; exit 1; }
  done
done
cd $R
for lab in auto -1; do for name in FETCH_SIZE TCC_HIT_sum_TCC_MISS_sum; do python3 profiles/pmc_part.py $out/pmc_${lab}_$name 4 8; done; done
