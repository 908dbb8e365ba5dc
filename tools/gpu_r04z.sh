#!/bin/bash
# r04 session 8: the interchanges left of each block deferred to one final pass (N <= 2048):
# factor A/B against HEAD (fingerprints must match), Stage-II tests, kernel stats of the new form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/lu_ab.py --libs variants/lu_head.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_head.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04z_lu_ab.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04z_lu_ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], round(r['best_ms'],2), round(r['frac_fp32_mfma'],3), r['lu_bits_sum'], r['piv_sum'], r['backward_error'], round(min(r['solve_ms']),3))"
bash tools/gpu_tests.sh r04z 900 tests/test_lu_hbm_gpu.py tests/test_stage2_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04z_prof -o lu -- python3 -u tools/lu_ab.py --child --batch 1024 --N 2000 --reps 2 > gpurun_out/r04z_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r04z_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r04z_lu_kernel_stats.csv; head -14 gpurun_out/r04z_lu_kernel_stats.csv | cut -c1-160
