#!/bin/bash
# r05: the CPU leg on all 64 of config 1's instances, once, beside one bench step
set -o pipefail
mkdir -p gpurun_out
( while true; do date >> gpurun_out/r05t_heartbeat.txt; sleep 30; done ) &
hb=$!
timeout -k 10 1000 python3 -u bench.py --cpu-sample 64 --steps 1 --warmup 1 --alt-f16x3 0 --train-batch 0 --stage2-iters 0 \
  > gpurun_out/r05_cpu_leg_64.json 2> gpurun_out/r05_cpu_leg_64.log
rc=$?
kill $hb
tail -c 800 gpurun_out/r05_cpu_leg_64.json
exit $rc
