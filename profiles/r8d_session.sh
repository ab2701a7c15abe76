#!/bin/bash
# round 4: hot-head count A/B at configs[2]'s size with the probe summary off (the new default):
# 262,144 heads (one per 512 handles, libfgi) / 524,288 / 1,048,576 / 2,097,152, two alternating rounds.
set -u
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r8d_ab27 2 --args --config rmat27 -- $L/libfgi.so $L/libfgi_hot524288d256.so $L/libfgi_hot1048576d128.so $L/libfgi_hot2097152d64.so || exit 1
