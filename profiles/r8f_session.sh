#!/bin/bash
# round 4: per-dispatch FETCH_SIZE / WRITE_SIZE / TCC hit-miss of configs[2]'s wave (R-MAT 27 on one GPU,
# profiles/wave_levels.py rmat27) with 524,288 hot heads, one counter group per rocprofv3 pass
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcl_r8f
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=2
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 200 rocprofv3 --pmc $pmc -T -d "$OUT/p$i" -o run --output-format csv -- \
        python3 "$R/profiles/wave_levels.py" rmat27 > "$OUT/p$i.out" 2> "$OUT/p$i.err" || exit 30
done
cd "$R" && python profiles/pmc_levels.py gpurun_out/pmcl_r8f > gpurun_out/pmcl_r8f/summary.txt && tail -60 gpurun_out/pmcl_r8f/summary.txt
