#!/bin/bash
# r05 session 1b: graph capture (info zeroed by a kernel), the x6 full-window gradients, K = 100 with the
# adopted epoch-55 checkpoint ("trained") beside e30
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -s \
  tests/test_abi_concurrency_gpu.py tests/test_train_window_gpu.py "tests/test_k100_gpu.py" \
  > gpurun_out/r05b_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05b_tests.log
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05b_tests.log | tail -30
exit $rc
