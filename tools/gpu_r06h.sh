#!/bin/bash
# r06: panels apply the previous panel's rank-16 update to their own columns (lu_panel_kernel PRE) --
# LU tests, A/B against HEAD's build (factors must be bitwise: same lu_bits_sum), LU profile (stats + PMC)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_stage2_gpu.py tests/test_abi_concurrency_gpu.py tests/test_lu_hbm_gpu.py > gpurun_out/r06h_lu_tests.log 2>&1 || { tail -n 40 gpurun_out/r06h_lu_tests.log; exit 1; }
tail -n 2 gpurun_out/r06h_lu_tests.log
timeout -k 10 600 python3 tools/lu_ab.py --libs tools/var_lu_head.so i-admm-lstm_amd/iadmm/libiadmm.so \
  tools/var_lu_head.so i-admm-lstm_amd/iadmm/libiadmm.so --batch 1024 --N 2000 > gpurun_out/r06h_lu_ab_pre.txt 2>&1 || exit 2
grep '^{' gpurun_out/r06h_lu_ab_pre.txt | cut -c1-130
bash tools/profile_lu.sh r06h 1024 2000 || exit 3
ls gpurun_out/prof_lu_r06h
