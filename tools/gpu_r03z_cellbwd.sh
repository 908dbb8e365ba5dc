#!/bin/bash
# Cell-backward A/B (in-tree vs a variant, bitwise checksums) + the training GPU tests.
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out/$tag
timeout -k 10 400 python3 tools/cellbwd_ab.py --libs "$@" > gpurun_out/$tag/cellbwd_ab.txt 2>&1 || exit 1
grep -o '"lib": "[^"]*"\|best_ms": [0-9.]*\|"checksums": \[[^]]*\]' gpurun_out/$tag/cellbwd_ab.txt | paste - - - | sed 's|/tmp/code/[^ ]*repo/||'
bash tools/gpu_tests.sh ${tag}_train 600 tests/test_train_gpu.py tests/test_train_config5_gpu.py tests/test_train_split_gpu.py tests/test_metric_grad_gpu.py || exit 1
