#!/bin/bash
# One GPU-box measurement session (repo root): per-level phase probes of the configs[1] wave,
# bench_configs.py (configs[0], [3], [4]) and a kernel trace of the configs[3] churn + prune.
# Stops at the first failing step. Usage: profiles/measure_session.sh <tag>
#   SKIP_PROBE=1 / SKIP_CONFIGS=1 / SKIP_PRUNE_TRACE=1 skip those steps.
TAG=${1:-m}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
if [ "${SKIP_PROBE:-0}" != 1 ]; then
    FGI_LIBRARY=$R/stl.fusion_amd/lib/libfgi_probe.so FGI_TRACE=1 timeout -k 10 240 python -u profiles/wave_levels.py \
        > "$O/probe.log" 2>&1 || { echo "probe rc=$?"; exit 31; }
    grep -E "^\[probe\]|^wave" "$O/probe.log" | tail -20
fi
if [ "${SKIP_CONFIGS:-0}" != 1 ]; then
    timeout -k 10 600 python -u bench_configs.py $CONFIG_ARGS > "$O/configs.jsonl" 2> "$O/configs.err" \
        || { echo "configs rc=$?"; exit 32; }
    cat "$O/configs.jsonl"
fi
if [ "${SKIP_PRUNE_TRACE:-0}" != 1 ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$O/prune_trace" -o run --output-format csv -- \
        python3 "$R/bench_configs.py" --only churn --no-cpu --steps 3 > "$O/prune_trace.jsonl" 2> "$O/prune_trace.err" \
        || { echo "prune trace rc=$?"; exit 33; }
    echo "prune trace done"
fi
