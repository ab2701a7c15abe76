#!/bin/bash
# round 4: threads per k_roots block (256 default; 128; 64: 4,096 roots in 16 / 32 / 64 blocks), configs[1]
set -u
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r8p_ab24 3 $L/libfgi.so $L/libfgi_rootblk128.so $L/libfgi_rootblk64.so || exit 1
