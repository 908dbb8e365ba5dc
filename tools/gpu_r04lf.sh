#!/bin/bash
# r04 session 8: the left pass of all but the last block beside the last block's factorization (low-priority stream), vs HEAD:
# factor A/B against HEAD (fingerprints must match), Stage-II tests, kernel stats of the new form
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/lu_ab.py --libs variants/lu_final.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_final.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04lf_lu_ab.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04lf_lu_ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], round(r['best_ms'],2), round(r['frac_fp32_mfma'],3), r['lu_bits_sum'], r['piv_sum'], r['backward_error'], round(min(r['solve_ms']),3))"
bash tools/gpu_tests.sh r04lf 900 tests/test_lu_hbm_gpu.py tests/test_stage2_gpu.py tests/test_k100_gpu.py tests/test_config4_gpu.py || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04lf_prof -o lu -- python3 -u tools/lu_ab.py --child --batch 1024 --N 2000 --reps 2 > gpurun_out/r04lf_prof.log 2>&1 || exit $?
f=$(find gpurun_out/r04lf_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r04lf_lu_kernel_stats.csv; rm -rf gpurun_out/r04lf_prof
python3 - gpurun_out/r04lf_lu_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "lu_" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>5s} total {float(r["TotalDurationNs"])/1e6:8.2f} ms avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
