#!/bin/bash
# r04 session 8: the default bench line at HEAD (LU with staged panels) (as the driver runs it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r04x_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r04x_bench.log > gpurun_out/r04x_bench.json
tail -c 3000 gpurun_out/r04x_bench.json
