#!/bin/bash
set -euo pipefail
export TMPDIR=/tmp
raw=$(mktemp -d /tmp/pt_XXXX)
mkdir -p gpurun_out/prof_train
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$raw" -o run -- python3 bench_train.py --batch 512 --micro_batch 128 --steps 1 --warmup 0 > gpurun_out/prof_train/log.txt 2>&1
cp "$(find "$raw" -name "*kernel_stats.csv" | head -1)" gpurun_out/prof_train/${TAG:-r02}_train_config5_B512_kernel_stats.csv
rm -rf "$raw"
