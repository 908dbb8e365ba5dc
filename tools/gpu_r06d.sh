#!/bin/bash
# r06: window gradient sums + one-round GEMM splits -- training tests, batch-2 / batch-32 windows, kernel
# trace of the batch-2 window; then the LU capture bisection on the guard-free variant (last: may crash)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_window_grads_gpu.py tests/test_train_gpu.py tests/test_train_window_gpu.py tests/test_train_config5_gpu.py \
  tests/test_train_split_gpu.py tests/test_metric_grad_gpu.py tests/test_dropin_gpu.py > gpurun_out/r06d_tests.log 2>&1 || { tail -n 40 gpurun_out/r06d_tests.log; exit 1; }
tail -n 3 gpurun_out/r06d_tests.log
timeout -k 10 300 python3 -u bench_train.py --batch 2 --micro_batch 2 --steps 5 --warmup 1 > gpurun_out/r06d_b2_bench.json 2> gpurun_out/r06d_b2_bench.err || exit 2
head -c 300 gpurun_out/r06d_b2_bench.json; echo
timeout -k 10 300 python3 -u bench_train.py --steps 2 --warmup 1 > gpurun_out/r06d_b32_bench.json 2> gpurun_out/r06d_b32_bench.err || exit 3
head -c 300 gpurun_out/r06d_b32_bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06d_prof -o b2 -- python3 bench_train.py --batch 2 --micro_batch 2 --steps 1 --warmup 1 > gpurun_out/r06d_b2_prof.log 2>&1 || exit 4
export IADMM_LIB_PATH=$PWD/tools/var_lu_capture.so
for c in "raw 300 4 4" "torch 300 4 4" "torch 1100 4 4" "raw 2500 4 0" "torch 2500 4 0"; do
  timeout -k 10 120 python3 -u tools/lu_capture_bisect.py $c >> gpurun_out/r06d_capture_bisect.log 2>&1
  rc=$?
  echo "case [$c] rc=$rc" >> gpurun_out/r06d_capture_bisect.log
  [ $rc -ne 0 ] && break
done
grep -v "amdgpu.ids" gpurun_out/r06d_capture_bisect.log | tail -30
exit 0
