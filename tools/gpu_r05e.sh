#!/bin/bash
# r05: the default bench line at HEAD (epoch-55 checkpoint, two-level LU, read-probe box ceiling)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/r05e_bench.json 2> gpurun_out/r05e_bench.log
rc=$?
tail -c 3000 gpurun_out/r05e_bench.json
exit $rc
