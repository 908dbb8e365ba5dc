#!/bin/bash
# r05: the 8-wave direct-accumulator paired update -- correctness, then default vs paired A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  "tests/test_stage2_gpu.py::test_paired_blocks_match_rank128_form" > gpurun_out/r05g_tests.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/r05g_tests.log
grep -E "PASSED|FAILED|ERROR|passed|failed|\[paired" gpurun_out/r05g_tests.log | tail -10
[ $rc -eq 0 ] || exit $rc
for fl in 0 2; do
  timeout -k 10 300 python -u tools/lu_ab.py --flags $fl --batch 1024 --N 2000 >> gpurun_out/r05g_lu_ab.txt 2>&1 || exit $?
done
grep best_ms gpurun_out/r05g_lu_ab.txt | python3 -c "import sys,json; [print(json.loads(l)['flags'], json.loads(l)['best_ms'], json.loads(l)['frac_fp32_mfma'], json.loads(l)['backward_error']) for l in sys.stdin]"
