#!/bin/bash
# r05: the two-workgroup rank-256 update -- breakdown, correctness of the paired path, default vs paired A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 ./tools/lubench256.bin > gpurun_out/r05j_lubench256.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_stage2_gpu.py::test_paired_blocks_match_rank128_form" > gpurun_out/r05j_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05j_tests.log
grep -E "PASSED|FAILED|ERROR|passed|failed|\[paired" gpurun_out/r05j_tests.log | tail -10
[ $rc -eq 0 ] || exit $rc
for fl in 0 2; do
  timeout -k 10 300 python -u tools/lu_ab.py --flags $fl --batch 1024 --N 2000 >> gpurun_out/r05j_lu_ab.txt 2>&1 || exit $?
done
grep best_ms gpurun_out/r05j_lu_ab.txt | python3 -c "import sys,json; [print(d['flags'], d['best_ms'], round(d['frac_fp32_mfma'],4), d['backward_error'], d['lu_bits_sum'], d['piv_sum']) for d in map(json.loads, sys.stdin)]"
