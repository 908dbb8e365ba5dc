#!/bin/bash
# r04 session 7: LU two-accumulator trailing update: speed A/B + backward error
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lu_ab.py --libs variants/lu_1acc.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_1acc.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04j_lu_ab_2acc.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04j_lu_ab_2acc.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], round(r['best_ms'],2), round(r['frac_fp32_mfma'],3), [round(x,3) for x in r['solve_ms'][:3]], r['backward_error'])"
timeout -k 10 400 python -u tools/lu_diag.py --N 2000 10000 --batch 2 > gpurun_out/r04j_lu_diag_2acc.log 2>&1 || exit $?
python3 - <<'PY'
import json
for line in open('gpurun_out/r04j_lu_diag_2acc.log'):
    if not line.startswith('{'): continue
    r=json.loads(line)
    h,m=r['hip_factor'],r['mkl_sgetrf']
    print(r['N'], r['instance'], 'hip %.2e (U12 %.2e L %.2e) mkl %.2e ratio %.2f' % (h['factor_berr'], h['R_U12'], h['R_L'], m['factor_berr'], h['factor_berr']/m['factor_berr']))
PY
