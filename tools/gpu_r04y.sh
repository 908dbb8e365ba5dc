#!/bin/bash
# r04 session 8: 1537-2048-row panels with two rows per thread in the LDS stage (one round):
# panel microbenchmark + determinism, factor A/B fingerprints, Stage-II tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 ./tools/lupanelbench.bin 1024 > gpurun_out/r04y_lupanelbench.txt 2>&1 || exit $?
grep -v "determinism" gpurun_out/r04y_lupanelbench.txt; grep "determinism" gpurun_out/r04y_lupanelbench.txt | grep -v " 0 differing matrix words, 0 differing pivots" ; grep -c " 0 differing matrix words, 0 differing pivots" gpurun_out/r04y_lupanelbench.txt
timeout -k 10 400 python -u tools/lu_ab.py --libs variants/lu_staged.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_staged.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04y_lu_ab.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04y_lu_ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], round(r['best_ms'],2), round(r['frac_fp32_mfma'],3), r['lu_bits_sum'], r['piv_sum'], r['backward_error'])"
bash tools/gpu_tests.sh r04y 900 tests/test_stage2_gpu.py tests/test_lu_hbm_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py || exit $?
