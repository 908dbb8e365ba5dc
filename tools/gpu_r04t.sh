#!/bin/bash
# r04 session 8: Stage II above the LDS limit (HBM solve, interchange pass) + the Stage-II suites
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh r04t 900 tests/test_lu_hbm_gpu.py tests/test_stage2_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py || exit $?
grep "lu hbm" gpurun_out/r04t_tests.log
