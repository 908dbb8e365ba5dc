#!/bin/bash
# r04 session 8: full -m gpu suite (one process) + smoke at HEAD
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_suite.sh r04h || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04h_smoke.log 2>&1 || exit $?
tail -2 gpurun_out/r04h_smoke.log
