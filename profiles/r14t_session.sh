#!/bin/bash
# Round 6: kernel trace of the bench's pipelined (asynchronous) leg, configs[1]: its waves' launch patterns and
# kernel times against the synchronous waves'
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14t; mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T -d $out/trace -o run --output-format csv -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu --no-e2e --no-secondary > $out/bench.json 2> $out/bench.err || { echo "rc=$?"; tail -5 $out/bench.err; exit 1; }
echo done
