#!/bin/bash
# LU / solve A/B on the GPU box: Stage-II GPU tests with the in-tree library, then factorization and
# solve times + backward error for each library build given (tools/lu_ab.py).
# Usage: bash tools/gpu_lu_ab.sh <tag> lib.so...
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
bash tools/gpu_tests.sh ${tag}_stage2 500 tests/test_stage2_gpu.py || exit 1
timeout -k 10 300 python3 tools/lu_ab.py --libs "$@" --batch 1024 --N 2000 > gpurun_out/$tag/lu_ab.txt 2>&1 || exit 1
grep lib gpurun_out/$tag/lu_ab.txt | cut -c1-400
