#!/bin/bash
# r04 session 8: Stage-II LU profile (trace + FETCH/WRITE passes) and training kernel trace at HEAD
set -o pipefail
mkdir -p gpurun_out
bash tools/profile_lu.sh r04 1024 2000 || exit $?
TAG=r04 bash tools/profile_train.sh || exit $?
ls gpurun_out/prof_lu_r04 gpurun_out/prof_train
