#!/bin/bash
# r04 session 8: f16x3 cell on the LDS-DMA ring: A/B vs the register-staged form, f16x3 tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/f16x3_ab.py --libs variants/f16x3_old.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04w_f16x3_ab.txt 2>&1 || exit $?
grep '^{' gpurun_out/r04w_f16x3_ab.txt | python3 -c "
import sys,json
for l in sys.stdin:
    r=json.loads(l); print(r['lib'].split('/')[-1], r.get('best_ms'), r.get('tflops_f32_equiv'), r.get('H_vs_fp32'), r.get('C_vs_fp32'), r.get('rc'))"
bash tools/gpu_tests.sh r04w 600 tests/test_f16x3_gpu.py tests/test_k100_gpu.py -k "f16x3" || exit $?
