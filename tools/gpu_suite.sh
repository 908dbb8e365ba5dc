#!/bin/bash
# The whole -m gpu suite in one process (as the driver runs it), log in gpurun_out/<tag>_gputest.log
set -o pipefail
tag=${1:-r03}
mkdir -p gpurun_out
timeout -k 10 1050 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread -s > "gpurun_out/${tag}_gputest.log" 2>&1
rc=$?
echo "rc=$rc" >> "gpurun_out/${tag}_gputest.log"
tail -3 "gpurun_out/${tag}_gputest.log"
exit $rc
