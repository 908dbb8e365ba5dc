#!/bin/bash
# Solve A/B: the Stage-II tests against a variant library, then lu_ab (factor + solve times, backward error).
# Usage: bash tools/gpu_r03z_solve.sh <tag> <variant.so> lib.so...
set -o pipefail
tag=$1; var=$2; shift 2
mkdir -p gpurun_out/$tag
IADMM_LIB_PATH=$(pwd)/$var bash tools/gpu_tests.sh ${tag}_stage2 500 tests/test_stage2_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py -k "stage2 or lu" || exit 1
timeout -k 10 400 python3 tools/lu_ab.py --libs "$@" --batch 1024 --N 2000 > gpurun_out/$tag/lu_ab.txt 2>&1 || exit 1
grep lib gpurun_out/$tag/lu_ab.txt | cut -c1-300
