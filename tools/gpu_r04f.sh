#!/bin/bash
# r04 session 6: cell-backward staged-dP A/B (determinism: checksums must equal the old build's) + training tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/cellbwd_ab.py --libs variants/cb_old.so i-admm-lstm_amd/iadmm/libiadmm.so > gpurun_out/r04i_cellbwd_stage_ab.txt 2>&1 || exit $?
grep -o '"lib": "[^"]*"\|best_ms": [0-9.]*\|"checksums": \[[^]]*\]' gpurun_out/r04i_cellbwd_stage_ab.txt | paste - - - | sed 's|/tmp/code/[^ ]*repo/||'
bash tools/gpu_tests.sh r04i 900 tests/test_train_config5_gpu.py tests/test_train_gpu.py tests/test_train_split_gpu.py tests/test_cell_gpu.py || exit $?
