#!/bin/bash
# r06: the default bench line at HEAD + its kernel stats under rocprofv3; then the FUSE variant's LU tests
# and A/B against the product (tools/gpu_r06j.sh)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06y}
timeout -k 10 600 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log || { tail -5 gpurun_out/${tag}_bench.log; exit 3; }
head -c 400 gpurun_out/${tag}_bench.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 --alt-f16x3 0 > gpurun_out/${tag}_bench_under_trace.json 2> gpurun_out/${tag}_prof.log || exit 4
bash tools/gpu_r06j.sh
