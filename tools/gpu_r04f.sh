#!/bin/bash
# r04 session 8, final state: Stage-II LU profile (kernel stats + FETCH/WRITE PMC passes, one
# factorization each), the whole -m gpu suite in one process, smoke
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_lu.sh r04c 1024 2000 || exit $?
bash tools/gpu_suite.sh r04f || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.log 2>&1 || exit $?
tail -3 gpurun_out/r04f_smoke.log
