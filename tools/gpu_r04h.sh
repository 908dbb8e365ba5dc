#!/bin/bash
# r04 session 8, final state (look-ahead, priorities, mid update in 70 KB, permutation in the L11^-1
# launch): Stage-II LU profile (kernel stats + FETCH/WRITE PMC passes, one factorization each), the
# whole -m gpu suite in one process, smoke
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_lu.sh r04d 1024 2000 || exit $?
bash tools/gpu_suite.sh r04h || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04h_smoke.log 2>&1 || exit $?
tail -3 gpurun_out/r04h_smoke.log
