#!/bin/bash
# round 4: final-collect / wave-init grid geometry A/B on configs[1] (libfgi: 1,024 final blocks of >= 256
# bitmap words, 512 init blocks), three alternating rounds on one box
set -u
L=stl.fusion_amd/lib
bash profiles/r5_ab.sh r8m_ab24 3 $L/libfgi.so $L/libfgi_grid2048_128_512.so $L/libfgi_grid1024_256_2048.so $L/libfgi_grid4096_64_2048.so || exit 1
