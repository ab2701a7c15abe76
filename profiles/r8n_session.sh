#!/bin/bash
# round 4: 16 KB LDS hot snapshot (131,072 heads in LDS, occupancy 4) against 8 KB (65,536, occupancy 5),
# configs[2]'s graph and configs[1], alternating
set -u
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r8n_ab27 2 --args --config rmat27 -- $L/libfgi.so $L/libfgi_ldshot4096.so || exit 1
bash profiles/r5_ab.sh r8n_ab24 2 $L/libfgi.so $L/libfgi_ldshot4096.so || exit 1
