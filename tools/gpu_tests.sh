#!/bin/bash
# Run a list of GPU test files on the box with a per-run time limit; log to gpurun_out/<tag>_tests.log.
# Usage: bash tools/gpu_tests.sh <tag> <limit_s> test_file...
set -o pipefail
tag=$1; lim=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 "$lim" python -u -m pytest -x -v --timeout "$lim" --timeout-method thread -s "$@" > "gpurun_out/${tag}_tests.log" 2>&1
rc=$?
echo "rc=$rc" >> "gpurun_out/${tag}_tests.log"
tail -4 "gpurun_out/${tag}_tests.log"
exit $rc
