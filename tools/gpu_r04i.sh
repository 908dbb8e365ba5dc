#!/bin/bash
# r04 session 8: forward cell A/B (direct vs LDS-staged whole-line H'/C' stores), bitwise check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 ./tools/cellbench.bin 1024 7 > gpurun_out/r04i_cellbench_stg.txt 2>&1 || exit $?
cat gpurun_out/r04i_cellbench_stg.txt | grep -v "^stamps"
