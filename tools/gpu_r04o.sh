#!/bin/bash
# r04 session 8: buffer soffset range-check probe; trailing update A/B r03 / paired / direct
set -o pipefail
mkdir -p gpurun_out
timeout -k 5 60 ./tools/buffer_soffset_probe.bin > gpurun_out/r04o_soffset_probe.txt 2>&1 || exit $?
cat gpurun_out/r04o_soffset_probe.txt
timeout -k 10 300 ./tools/lubench128.bin 1024 2000 > gpurun_out/r04o_lubench128.txt 2>&1 || exit $?
cat gpurun_out/r04o_lubench128.txt
