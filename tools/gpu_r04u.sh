#!/bin/bash
# r04 session 8: full -m gpu suite + smoke at HEAD, then the Stage-II LU profile (trace + FETCH/WRITE)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_suite.sh r04u || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04u_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r04u_smoke.log
bash tools/profile_lu.sh r04b 1024 2000 || exit $?
ls gpurun_out/prof_lu_r04b
