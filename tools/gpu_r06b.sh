#!/bin/bash
# r06: tests touched by the ADVICE fixes (two L11^-1 buffers, B=512 split vs rank-128); the batch-2 recipe
# window measured (wall, cProfile, rocprof kernel trace); the LU capture probe on the guard-free variant
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_abi_concurrency_gpu.py "tests/test_stage2_gpu.py::test_paired_blocks_match_rank128_form" \
  tests/test_train_gpu.py > gpurun_out/r06b_tests.log 2>&1 || { tail -n 30 gpurun_out/r06b_tests.log; exit 1; }
tail -n 3 gpurun_out/r06b_tests.log
timeout -k 10 300 python3 -u bench_train.py --batch 2 --micro_batch 2 --steps 3 --warmup 1 > gpurun_out/r06b_b2_bench.json 2> gpurun_out/r06b_b2_bench.err || exit 2
head -c 600 gpurun_out/r06b_b2_bench.json; echo
timeout -k 10 300 python3 -u -m cProfile -o gpurun_out/r06b_b2.prof bench_train.py --batch 2 --micro_batch 2 --steps 1 --warmup 1 > /dev/null 2>&1 || exit 3
python3 -c "import pstats; pstats.Stats('gpurun_out/r06b_b2.prof').sort_stats('tottime').print_stats(25)" > gpurun_out/r06b_b2_cprofile.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06b_prof -o b2 -- python3 bench_train.py --batch 2 --micro_batch 2 --steps 1 --warmup 1 > gpurun_out/r06b_b2_prof.log 2>&1 || exit 4
find gpurun_out/r06b_prof -name "*stats*" | head
IADMM_LIB_PATH=$PWD/tools/var_lu_capture.so timeout -k 10 300 python3 -u tools/lu_capture_probe.py > gpurun_out/r06b_capture_probe.log 2>&1
rc=$?
cat gpurun_out/r06b_capture_probe.log | tail -20
exit $rc
