#!/bin/bash
# r05: paired-update main-loop variants (lu_trail256_kernel<MODE>, experiment flag bits 4/8):
# 0 = drain + issue + chain + store per step; 1 = the drain leaves the last stores in flight;
# 2 = memory work interleaved in the chain, three accumulator sets; 3 = 2 with asm fragment reads.
# One factorization fingerprint per mode (identical arithmetic: must agree) and the factor time.
set -o pipefail
mkdir -p gpurun_out
for fl in 0 2 6 10 14; do
  timeout -k 10 300 python -u tools/lu_ab.py --flags $fl --batch 1024 --N 2000 >> gpurun_out/r05h_lu_ab.txt 2>&1 || exit $?
done
grep best_ms gpurun_out/r05h_lu_ab.txt | python3 -c "import sys,json; [print(d['flags'], d['best_ms'], round(d['frac_fp32_mfma'],4), d['backward_error'], d['lu_bits_sum'], d['piv_sum']) for d in map(json.loads, sys.stdin)]"
