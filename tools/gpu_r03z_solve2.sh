#!/bin/bash
# Solve thread-count A/B: Stage-II tests (small batches take the 1024-thread solve), then config-4
# Stage II with the in-tree build and with variants/prev.so (256-thread solve only).
set -o pipefail
mkdir -p gpurun_out/r03z9
bash tools/gpu_tests.sh r03z9_stage2 500 tests/test_stage2_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py -k "stage2 or lu" || exit 1
for lib in i-admm-lstm_amd/iadmm/libiadmm.so variants/prev.so; do
  tagl=$(basename $lib .so)
  IADMM_LIB_PATH=$(pwd)/$lib timeout -k 10 500 python3 -u bench_stage2.py --batch 512 --num_var 5000 --num_ineq 2500 --num_eq 2500 \
    --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/r03z9/stage2_config4_$tagl.json 2> gpurun_out/r03z9/stage2_config4_$tagl.err || exit 1
  grep '^{' gpurun_out/r03z9/stage2_config4_$tagl.json | cut -c1-300
done
