#!/bin/bash
# r03 session 2: Stage-II tests, LU A/B of library builds, LU kernel profile of the in-tree build.
# Usage: bash tools/gpu_r03z.sh <tag> lib.so...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
bash tools/gpu_lu_ab.sh $tag "$@" || exit 1
bash tools/profile_lu.sh $tag > gpurun_out/$tag/profile.log 2>&1 || exit 1
echo done
