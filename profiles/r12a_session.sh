#!/bin/bash
# Round 5 (after the fold rewrite): rocprofv3 evidence for HEAD — kernel trace + separate PMC passes of configs[1] (R-MAT 24) and
# configs[2] (R-MAT 27) headline runs, then bench.py --gpus 2 as two processes on this one GPU (host
# collectives over gloo: the N > 1 path end to end).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r12a; mkdir -p $out
bash profiles/run_profile.sh r12c1 --config rmat24 --no-secondary --no-cpu --no-e2e --steps 10 --warmup 2 > $out/prof_c1.log 2>&1 || { echo "profile c1 rc=$?"; tail -20 $out/prof_c1.log; exit 1; }
bash profiles/run_profile.sh r12c2 --config rmat27 --no-secondary --no-cpu --no-e2e --steps 10 --warmup 2 > $out/prof_c2.log 2>&1 || { echo "profile c2 rc=$?"; tail -20 $out/prof_c2.log; exit 1; }
echo "profiles done"
cd $R
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 3 --warmup 1 > $out/bench_n2_host.json 2> $out/bench_n2_host.err || { echo "n2 bench rc=$?"; tail -30 $out/bench_n2_host.err; exit 1; }
cat $out/bench_n2_host.json | cut -c1-1500
