#!/bin/bash
# round 6: 4 KiB / 8 KiB kernels at enforced residencies (LDS granules fixed) and grid rounds
set -e
bash tools/ab_tune.sh ". .:waves_per_simd=3 .:waves_per_simd=3,grid_rounds=1 .:waves_per_simd=4,grid_rounds=2 .:waves_per_simd=4,grid_rounds=8" udp64 vxlan 2>&1 | tee gpurun_out/ab_w3.txt
