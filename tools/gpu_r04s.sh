#!/bin/bash
# r04 session 8: staged panels (drained stores): factor A/B fingerprints (two runs each) + Stage-II / K=100 / config-4 tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/lu_ab.py --libs variants/lu_paired.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_paired.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04s_lu_ab.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04s_lu_ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], round(r['best_ms'],2), round(r['frac_fp32_mfma'],3), r['lu_bits_sum'], r['piv_sum'], r['backward_error'])"
bash tools/gpu_tests.sh r04s 900 tests/test_stage2_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py tests/test_dropin_gpu.py || exit $?
