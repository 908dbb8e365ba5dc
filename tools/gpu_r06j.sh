#!/bin/bash
# r06: in-half updates inside the panels (lu_panel_kernel FUSE, built as tools/var_lu_fuse.so) -- LU
# tests on the variant, A/B against the product build (PRE; factors must be bitwise: same lu_bits_sum)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
IADMM_LIB_PATH=$PWD/tools/var_lu_fuse.so timeout -k 10 900 python3 -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_stage2_gpu.py tests/test_abi_concurrency_gpu.py tests/test_lu_hbm_gpu.py > gpurun_out/r06j_lu_tests.log 2>&1 || { tail -n 40 gpurun_out/r06j_lu_tests.log; exit 1; }
tail -n 2 gpurun_out/r06j_lu_tests.log
timeout -k 10 600 python3 tools/lu_ab.py --libs i-admm-lstm_amd/iadmm/libiadmm.so tools/var_lu_fuse.so \
  i-admm-lstm_amd/iadmm/libiadmm.so tools/var_lu_fuse.so --batch 1024 --N 2000 > gpurun_out/r06j_lu_ab_fuse.txt 2>&1 || exit 2
grep '^{' gpurun_out/r06j_lu_ab_fuse.txt | cut -c1-130
