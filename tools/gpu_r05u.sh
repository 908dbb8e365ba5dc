#!/bin/bash
# r05: the K = 100 fp64-envelope test over the committed weights and every candidate (incl. the new e61)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -s tests/test_k100_gpu.py \
  > gpurun_out/r05u_k100.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05u_k100.log
grep -E "worst distance|PASSED|FAILED|passed|failed" gpurun_out/r05u_k100.log | cut -c1-250 | tail -14
exit $rc
