#!/bin/bash
# r06: small-M GEMM splits (gemm_nt over K, gemm_tn rows by fill) -- training tests, batch-2 and batch-32
# windows, a kernel trace of the batch-2 window; then the capture probe variants (last: may crash)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_train_gpu.py tests/test_train_window_gpu.py tests/test_train_config5_gpu.py tests/test_train_split_gpu.py \
  tests/test_metric_grad_gpu.py > gpurun_out/r06c_tests.log 2>&1 || { tail -n 40 gpurun_out/r06c_tests.log; exit 1; }
tail -n 3 gpurun_out/r06c_tests.log
timeout -k 10 300 python3 -u bench_train.py --batch 2 --micro_batch 2 --steps 5 --warmup 1 > gpurun_out/r06c_b2_bench.json 2> gpurun_out/r06c_b2_bench.err || exit 2
head -c 300 gpurun_out/r06c_b2_bench.json; echo
timeout -k 10 300 python3 -u bench_train.py --steps 2 --warmup 1 > gpurun_out/r06c_b32_bench.json 2> gpurun_out/r06c_b32_bench.err || exit 3
head -c 300 gpurun_out/r06c_b32_bench.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06c_prof -o b2 -- python3 bench_train.py --batch 2 --micro_batch 2 --steps 1 --warmup 1 > gpurun_out/r06c_b2_prof.log 2>&1 || exit 4
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/capture_probe.hip -o /tmp/capture_probe || exit 5
for v in 1 2 3 4 5 6 7 8; do
  timeout -k 10 60 /tmp/capture_probe $v >> gpurun_out/r06c_capture_probe.log 2>&1
  rc=$?
  echo "variant $v rc=$rc" >> gpurun_out/r06c_capture_probe.log
  [ $rc -ne 0 ] && break
done
cat gpurun_out/r06c_capture_probe.log | tail -30
exit 0
