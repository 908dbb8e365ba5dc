#!/bin/bash
# r03r: the f16x3 K=100 oracle test, then Stage II at the config-4 shape (bench_stage2.py).
set -o pipefail
mkdir -p gpurun_out/r03r
bash tools/gpu_tests.sh r03r_f16x3 500 tests/test_k100_gpu.py -k f16x3 || exit 1
timeout -k 10 500 python3 -u bench_stage2.py --batch 512 --num_var 5000 --num_ineq 2500 --num_eq 2500 \
  --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/r03r/stage2_config4.json 2> gpurun_out/r03r/stage2_config4.err || exit 1
grep '^{' gpurun_out/r03r/stage2_config4.json | cut -c1-700
