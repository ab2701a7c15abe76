#!/bin/bash
# Hot-heads snapshot size A/B (64 Ki default vs 256 Ki vs 1 Mi heads) on configs[1] (rmat24) and at
# scale 27, where the scale-27 level counters (r5d_pmc_levels_rmat27.txt) show 23 % L2 hits on the
# L1 pull level.
set -u
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r5e_ab24 2 $L/libfgi.so $L/libfgi_hot262144.so $L/libfgi_hot1048576.so || exit 1
bash profiles/r5_ab.sh r5e_ab27 2 --args --config rmat27 -- $L/libfgi.so $L/libfgi_hot262144.so $L/libfgi_hot1048576.so || exit 1
