#!/bin/bash
# Round 6, final profiles: rocprofv3 kernel trace + stats and the PMC passes (FETCH_SIZE, WRITE_SIZE, L2 hit/miss,
# atomics; one pass each) of the bench's synchronous timed waves, configs[1] (r14p1) and configs[2] on one GPU
# (r14p2); summarised (in the container, after the merge) into profiles/r14p{1,2}_summary.json by profiles/summarize.py (bench.py's roofline traffic)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash profiles/run_profile.sh r14p1 --steps 10 --warmup 2 --no-cpu --no-e2e --no-pipelined --no-secondary || { echo "profile r14p1 rc=$?"; exit 1; }
bash profiles/run_profile.sh r14p2 --config rmat27 --steps 5 --warmup 2 --no-cpu --no-e2e --no-pipelined --no-secondary || { echo "profile r14p2 rc=$?"; exit 1; }
echo "profiles done (summarise here: python3 profiles/summarize.py gpurun_out/prof_r14p1 r14p1 --steps 10, r14p2 --steps 5)"
