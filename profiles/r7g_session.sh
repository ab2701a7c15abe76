#!/bin/bash
# round 4: GPU suite, then the headline bench with fused waves and without (A/B on one box)
set -e
out=gpurun_out/${1:-r7g}
mkdir -p $out
timeout -k 10 480 python -u -m pytest -x -q --durations=15 --timeout 150 --timeout-method thread -m gpu tests > $out/gpu_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > $out/bench.json 2> $out/bench.err
FGI_FUSED=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $out/bench_nofuse.json 2> $out/bench_nofuse.err
FGI_FUSED_BLOCKS=128 timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $out/bench_fb128.json 2> $out/bench_fb128.err
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-e2e > $out/bench2.json 2> $out/bench2.err
