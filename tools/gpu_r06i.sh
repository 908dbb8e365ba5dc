#!/bin/bash
# r06: clean per-kernel LU durations: N = 2000, B = 1024 on one stream (no look-ahead / split), and the
# config-4 shape N = 10000, B = 256 (one chunk) as it runs by default (rank-128 blocks + look-ahead)
set -o pipefail
mkdir -p gpurun_out/r06i
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i/n2000 -o run -- \
  python3 tools/profile_lu.py --batch 1024 --N 2000 --no-lookahead > gpurun_out/r06i/n2000.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i/n10000 -o run -- \
  python3 tools/profile_lu.py --batch 256 --N 10000 > gpurun_out/r06i/n10000.log 2>&1 || exit 2
find gpurun_out/r06i -name "*kernel_stats.csv"
