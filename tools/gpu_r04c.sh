#!/bin/bash
# r04 session 3: LU ws microbench (LDS-DMA L21), LU factor A/B (ws wired vs not), cell-backward
# LDS-DMA epilogue A/B, MFMA rounding probe, LU diagnosis with fmaf
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 ./tools/mfma_fma_check.bin > gpurun_out/r04f_mfma_fma_check.txt 2>&1 || exit $?
cat gpurun_out/r04f_mfma_fma_check.txt
timeout -k 10 120 ./tools/lubench128.bin > gpurun_out/r04f_lubench128_ws.txt 2>&1 || exit $?
cat gpurun_out/r04f_lubench128_ws.txt
timeout -k 10 300 python -u tools/lu_ab.py --libs variants/lu_nows.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_nows.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04f_lu_ab_ws.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04f_lu_ab_ws.txt | cut -c1-330
timeout -k 10 400 python -u tools/cellbwd_ab.py --libs variants/cb_old.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04f_cellbwd_ldsdma_ab.txt 2>&1 || exit $?
grep -o '"lib": "[^"]*"\|best_ms": [0-9.]*\|"checksums": \[[^]]*\]' gpurun_out/r04f_cellbwd_ldsdma_ab.txt | paste - - - | sed 's|/tmp/code/[^ ]*repo/||'
timeout -k 10 400 python -u tools/lu_diag.py --N 2000 10000 --batch 2 > gpurun_out/r04f_lu_diag_fma.log 2>&1 || exit $?
