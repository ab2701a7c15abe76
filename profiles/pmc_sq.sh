#!/bin/bash
# Instruction-mix PMC pass (SQ counters, one pass) over a short bench run: per-dispatch instruction
# and cycle counts, used to find latency-bound launches. Usage: profiles/pmc_sq.sh <tag> [bench args]
TAG=${1:-sq}; shift
ARGS=${@:-"--steps 3 --warmup 1 --no-cpu"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -T -d "$OUT/pmc" -o run --output-format csv -- python3 "$R/bench.py" $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
