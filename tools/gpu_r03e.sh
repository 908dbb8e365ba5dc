#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r03e
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s "tests/test_k100_gpu.py::test_stage2_after_k100_vs_oracle" > gpurun_out/r03e/new.log 2>&1
echo "new rc=$?"; grep -E "stage2 N=2000|passed|failed" gpurun_out/r03e/new.log | cut -c1-330
IADMM_LIB_PATH=$PWD/variants/lu64.so timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread -s "tests/test_k100_gpu.py::test_stage2_after_k100_vs_oracle" > gpurun_out/r03e/old.log 2>&1
echo "old rc=$?"; grep -E "stage2 N=2000|passed|failed" gpurun_out/r03e/old.log | cut -c1-330
