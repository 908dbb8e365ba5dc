#!/bin/bash
# r03j: LU gathered-permutation + interleaved trailing update: Stage-II GPU tests, then A/B
# (factorization time, backward error) against the pre-change build and the trail microbenchmark.
set -o pipefail
mkdir -p gpurun_out/r03j
bash tools/gpu_tests.sh r03j_stage2 500 tests/test_stage2_gpu.py || exit 1
timeout -k 10 300 python3 tools/lu_ab.py --libs variants/base.so variants/g3.so variants/g4.so variants/g5.so --batch 1024 --N 2000 > gpurun_out/r03j/lu_ab.txt 2>&1 || exit 1
cat gpurun_out/r03j/lu_ab.txt
for v in g3 g4; do
  timeout -k 10 120 ./tools/lubench128_$v.bin 1024 2000 > gpurun_out/r03j/lubench128_$v.txt 2>&1 || exit 1
done
head -20 gpurun_out/r03j/lubench128_*.txt
