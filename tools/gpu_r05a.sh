#!/bin/bash
# r05 session 1: the new contract / parity tests (K = 100 fp64 envelope over every weight set,
# full-window training gradients, the HBM-form flag, Stage II with the two-level U12, ABI concurrency
# + graph capture + determinism) and the LU factor A/B against the r04 build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lu_ab.py --libs variants/lu_r04.so i-admm-lstm_amd/iadmm/libiadmm.so --batch 1024 --N 2000 \
  > gpurun_out/r05a_lu_ab.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/lu_ab.py --libs variants/lu_r04.so i-admm-lstm_amd/iadmm/libiadmm.so --batch 256 --N 10000 --reps 2 \
  >> gpurun_out/r05a_lu_ab.txt 2>&1 || exit $?
grep best_ms gpurun_out/r05a_lu_ab.txt | python3 -c "import sys,json; [print(json.loads(l)['lib'][-30:], json.loads(l)['best_ms']) for l in sys.stdin]"
timeout -k 10 1000 python -u -m pytest -v --timeout 900 --timeout-method thread -s \
  tests/test_probe_gpu.py tests/test_stage2_gpu.py tests/test_lu_hbm_gpu.py tests/test_train_window_gpu.py tests/test_k100_gpu.py \
  "tests/test_config4_gpu.py::test_config4_stage2_vs_oracle" tests/test_abi_concurrency_gpu.py \
  > gpurun_out/r05a_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05a_tests.log
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/r05a_tests.log | tail -40
exit $rc
