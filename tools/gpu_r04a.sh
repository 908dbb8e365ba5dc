#!/bin/bash
# r04 session 1: LU ws microbench, cell-backward persistent A/B, Stage-II blame attribution
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/lubench128.bin > gpurun_out/r04d_lubench128_ws.txt 2>&1 || exit $?
timeout -k 10 400 python -u tools/cellbwd_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so variants/cb_p1.so variants/cb_p1d4k.so variants/cb_p1d8k.so variants/cb_p1s8k.so variants/cb_p1s17k.so > gpurun_out/r04d_cellbwd_persist_ab.txt 2>&1 || exit $?
timeout -k 10 500 python -u tools/stage2_blame.py --n 5000 --batch 3 --iters 5 > gpurun_out/r04c_blame_N10000.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/stage2_blame.py --n 1000 --hidden 800 --length 100 --batch 4 --iters 5 > gpurun_out/r04c_blame_N2000.log 2>&1 || exit $?
cat gpurun_out/r04d_lubench128_ws.txt
grep '^{' gpurun_out/r04d_cellbwd_persist_ab.txt | cut -c1-200
