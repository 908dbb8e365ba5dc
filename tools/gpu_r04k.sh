#!/bin/bash
# r04 session 8: trailing update A/B: production (8 waves, 1 WG/CU) vs paired (4 waves, 2 WG/CU)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/lubench128.bin 1024 2000 > gpurun_out/r04k_lubench128_paired.txt 2>&1 || exit $?
cat gpurun_out/r04k_lubench128_paired.txt
