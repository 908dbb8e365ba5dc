#!/bin/bash
# r04 session 5: cell-backward staged-dP A/B, LU (fmaf + DPP argmax + readlane solve) A/B, training tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q -s tests/test_probe_gpu.py > gpurun_out/r04h_probe.log 2>&1; grep "box ceiling" gpurun_out/r04h_probe.log
timeout -k 10 400 python -u tools/cellbwd_ab.py --libs variants/cb_old.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04h_cellbwd_stage_ab.txt 2>&1 || exit $?
grep -o '"lib": "[^"]*"\|best_ms": [0-9.]*\|"checksums": \[[^]]*\]' gpurun_out/r04h_cellbwd_stage_ab.txt | paste - - - | sed 's|/tmp/code/[^ ]*repo/||'
timeout -k 10 300 python -u tools/lu_ab.py --libs variants/lu_nows.so i-admm-lstm_amd/iadmm/libiadmm.so variants/lu_nows.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04h_lu_ab_dpp.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04h_lu_ab_dpp.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], round(r['best_ms'],2), [round(x,3) for x in r['solve_ms'][:3]], r['lu_bits_sum'], r['piv_sum'])"
bash tools/gpu_tests.sh r04h 900 tests/test_train_config5_gpu.py tests/test_train_gpu.py tests/test_cell_gpu.py || exit $?
timeout -k 10 400 python -u tools/lu_diag.py --N 2000 10000 --batch 2 > gpurun_out/r04h_lu_diag_split.log 2>&1 || exit $?
