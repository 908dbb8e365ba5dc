#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03d
bash tools/gpu_tests.sh r03d 600 tests/test_stage2_gpu.py || exit 1
timeout -k 10 120 ./tools/lubench128.bin 1024 2000 > gpurun_out/r03d/lubench128.txt 2>&1 || exit 1
cat gpurun_out/r03d/lubench128.txt
timeout -k 10 400 python3 -u tools/lu_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so variants/lu128_v2.so variants/lu64.so --batch 1024 --N 2000 \
  > gpurun_out/r03d/lu_ab.txt 2>&1 || exit 1
grep '^{' gpurun_out/r03d/lu_ab.txt | cut -c1-250
