#!/bin/bash
# r05: last HEAD check (epoch-61 weights, batch-split LU, hoisted prologue loads) -- rank-256 breakdown, the whole -m gpu suite, smoke, the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/lubench256.bin > gpurun_out/r05ab_lubench256.txt 2>&1 || exit $?
bash tools/gpu_suite.sh r05ab || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05ab_smoke.log 2>&1 || exit $?
timeout -k 10 900 python3 -u bench.py > gpurun_out/r05ab_bench.json 2> gpurun_out/r05ab_bench.log
rc=$?
tail -c 1500 gpurun_out/r05ab_bench.json
exit $rc
