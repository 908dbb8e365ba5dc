#!/bin/bash
# r06: the restored x20 T=100 window-gradient case (measured chaos bound) and the bench-shape LU repeat test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread \
  tests/test_abi_concurrency_gpu.py::test_lu_bench_shape_repeat_bitwise \
  tests/test_train_window_gpu.py > gpurun_out/r06a_tests.log 2>&1
rc=$?
tail -n 40 gpurun_out/r06a_tests.log
exit $rc
