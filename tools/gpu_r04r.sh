#!/bin/bash
# r04 session 8: panel staging determinism: lgkmcnt-separated stores vs fully drained stores
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 ./tools/lupanelbench.bin 1024 > gpurun_out/r04r_lupanelbench.txt 2>&1 || exit $?
cat gpurun_out/r04r_lupanelbench.txt
timeout -k 10 240 ./tools/lupanelbench_drain.bin 1024 > gpurun_out/r04r_lupanelbench_drain.txt 2>&1 || exit $?
cat gpurun_out/r04r_lupanelbench_drain.txt
