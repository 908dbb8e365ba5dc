#!/bin/bash
# r05 session 2: paired blocks (rank-256 far update) -- correctness first, then the factor A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_stage2_gpu.py::test_paired_blocks_match_rank128_form" tests/test_stage2_gpu.py tests/test_lu_hbm_gpu.py \
  tests/test_abi_concurrency_gpu.py > gpurun_out/r05c_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05c_tests.log
grep -E "PASSED|FAILED|ERROR|passed|failed|\[paired" gpurun_out/r05c_tests.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/lu_ab.py --libs variants/lu_r04.so i-admm-lstm_amd/iadmm/libiadmm.so --batch 1024 --N 2000 \
  > gpurun_out/r05c_lu_ab.txt 2>&1 || exit $?
grep best_ms gpurun_out/r05c_lu_ab.txt | python3 -c "import sys,json; [print(json.loads(l)['lib'][-30:], json.loads(l)['best_ms'], json.loads(l)['frac_fp32_mfma']) for l in sys.stdin]"
