#!/bin/bash
# r03: LU tests with the fused half kernel, then the LU A/B (fused+rank128 / rank128 unfused / r02 flow)
set -o pipefail
bash tools/gpu_tests.sh r03b 600 tests/test_stage2_gpu.py tests/test_metric_grad_gpu.py tests/test_cell_gpu.py || exit 1
timeout -k 10 400 python3 -u tools/lu_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so variants/lu128_unfused.so variants/lu64.so \
  --batch 1024 --N 2000 > gpurun_out/r03b_lu_ab.txt 2>&1
echo "lu_ab rc=$?"; cat gpurun_out/r03b_lu_ab.txt | grep '^{'
