#!/bin/bash
# r04 session 8: profiles at HEAD: Stage-II LU (trace + FETCH/WRITE), bench kernel trace + PMC passes
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_lu.sh r04 1024 2000 || exit $?
bash tools/profile_bench.sh r04 || exit $?
ls gpurun_out/prof_lu_r04 gpurun_out/prof_r04/summary
