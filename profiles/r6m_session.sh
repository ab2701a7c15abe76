#!/bin/bash
# configs[3]'s prune under rocprofv3 from a torch-free process (profiles/prune_pmc.py): kernel trace,
# then one PMC pass per counter group for the fast path and FETCH_SIZE for the gather path. Any
# non-zero exit ends the call (the exit-time fault seen with torch in the process would show here).
set -u
R=$(pwd)
out=$R/gpurun_out/r6m
mkdir -p "$out"
export FGI_RESET_AT_EXIT=1   # r6m's first call: without it the profiled process faults in exit()
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
    python3 "$R/profiles/prune_pmc.py" > "$out/trace.json" 2> "$out/trace.err"
rc=$?; echo "trace rc=$rc"; cat "$out/trace.json"; [ $rc -eq 0 ] || exit $rc
for pmc in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo "$pmc" | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --pmc $pmc -d "$out/pmc_$name" -o run --output-format csv -- \
      python3 "$R/profiles/prune_pmc.py" > "$out/pmc_$name.json" 2> "$out/pmc_$name.err"
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
FGI_PRUNE_GATHER=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d "$out/pmc_gather_FETCH_SIZE" -o run --output-format csv -- \
    python3 "$R/profiles/prune_pmc.py" > "$out/pmc_gather_FETCH_SIZE.json" 2> "$out/pmc_gather_FETCH_SIZE.err"
rc=$?; echo "pmc gather FETCH_SIZE rc=$rc"; exit $rc
