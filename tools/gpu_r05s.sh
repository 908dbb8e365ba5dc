#!/bin/bash
# r05: config 4 at HEAD (tools/profile_config4.sh: PMC passes, the K=200 bench step, Stage II), with a
# heartbeat file so that the long steps show progress
set -o pipefail
mkdir -p gpurun_out/r05_cfg4
( while true; do date >> gpurun_out/r05_cfg4/heartbeat.txt; sleep 30; done ) &
hb=$!
bash tools/profile_config4.sh r05
rc=$?
kill $hb
tail -c 600 gpurun_out/r05_cfg4/bench_config4.json
tail -c 600 gpurun_out/r05_cfg4/stage2_config4.json
exit $rc
