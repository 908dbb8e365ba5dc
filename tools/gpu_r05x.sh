#!/bin/bash
# r05: batch split of the paired LU over the context's two streams -- Stage-II / ABI / HBM tests, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_stage2_gpu.py tests/test_abi_concurrency_gpu.py tests/test_lu_hbm_gpu.py > gpurun_out/r05x_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05x_tests.log
grep -E "passed|failed|FAILED|ERROR" gpurun_out/r05x_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for fl in 0 4; do
  timeout -k 10 300 python -u tools/lu_ab.py --flags $fl --batch 1024 --N 2000 >> gpurun_out/r05x_lu_ab.txt 2>&1 || exit $?
done
grep best_ms gpurun_out/r05x_lu_ab.txt | python3 -c "import sys,json; [print(d['flags'], d['best_ms'], round(d['frac_fp32_mfma'],4), d['backward_error'], d['lu_bits_sum'], d['piv_sum']) for d in map(json.loads, sys.stdin)]"
