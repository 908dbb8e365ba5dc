#!/bin/bash
# r04 session 2: MFMA rounding probe, LU ws microbench (deeper prefetch), LU diagnosis with fmaf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/mfma_fma_check.bin > gpurun_out/r04e_mfma_fma_check.txt 2>&1 || exit $?
timeout -k 10 120 ./tools/lubench128.bin > gpurun_out/r04e_lubench128_ws2.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/lu_diag.py --N 2000 10000 --batch 2 > gpurun_out/r04e_lu_diag_fma.log 2>&1 || exit $?
cat gpurun_out/r04e_mfma_fma_check.txt gpurun_out/r04e_lubench128_ws2.txt
timeout -k 10 300 python -u tools/lu_ab.py --libs variants/lu_nows.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_nows.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04e_lu_ab_ws.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04e_lu_ab_ws.txt | cut -c1-330
