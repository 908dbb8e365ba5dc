#!/bin/bash
# r05: prologue A12 gathers hoisted in lu_trail256_kernel -- Stage-II tests, then A/B against the HEAD build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_stage2_gpu.py tests/test_abi_concurrency_gpu.py > gpurun_out/r05aa_tests.log 2>&1 || { tail -5 gpurun_out/r05aa_tests.log; exit 1; }
tail -1 gpurun_out/r05aa_tests.log
for r in 1 2; do
  timeout -k 10 600 python -u tools/lu_ab.py --libs variants/lu_head.so i-admm-lstm_amd/iadmm/libiadmm.so --batch 1024 --N 2000 >> gpurun_out/r05aa_lu_ab.txt 2>&1 || exit $?
done
grep best_ms gpurun_out/r05aa_lu_ab.txt | python3 -c "import sys,json; [print(d['lib'][-30:], d['best_ms'], d['lu_bits_sum'], d['piv_sum']) for d in map(json.loads, sys.stdin)]"
