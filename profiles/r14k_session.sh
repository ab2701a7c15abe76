#!/bin/bash
# Round 6: bench.py --gpus 2 on a one-GPU box (2 ranks share the device, host collectives) with partition
# codes: configs[2]'s V_inv; level-1 FETCH per rank with the shipping (dealt) codes against none
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r14k; mkdir -p $out
cd $R
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-e2e --no-secondary > $out/bench_n2.json 2> $out/bench_n2.err || { echo "bench rc=$?"; tail -20 $out/bench_n2.err; exit 1; }
cat $out/bench_n2.json
cd /tmp && export TMPDIR=/tmp
for lab in auto -1; do
  env FGI_LABELS=$([ $lab = auto ] && echo 0 || echo -1) timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $out/pmc_${lab} -o run --output-format csv -- \
      python3 $R/profiles/part_local_timing.py 27 8 1 8 > $out/pmc_${lab}.out 2> $out/pmc_${lab}.err || { echo "pmc rc=$?"; exit 1; }
done
cd $R
for lab in auto -1; do python3 profiles/pmc_part.py $out/pmc_${lab} 4 8; done
