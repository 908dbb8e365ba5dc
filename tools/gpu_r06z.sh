#!/bin/bash
# r06 final HEAD check (as the driver runs it): the whole -m gpu suite, smoke, the default bench line,
# then the bench's kernel stats under rocprofv3 (profiles/)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-r06z}
bash tools/gpu_suite.sh $tag || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { tail -5 gpurun_out/${tag}_smoke.log; exit 2; }
tail -2 gpurun_out/${tag}_smoke.log
timeout -k 10 900 python3 -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log || { tail -5 gpurun_out/${tag}_bench.log; exit 3; }
head -c 700 gpurun_out/${tag}_bench.json; echo
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o bench -- python3 bench.py --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/${tag}_bench_under_trace.json 2> gpurun_out/${tag}_prof.log || exit 4
find gpurun_out/${tag}_prof -name "*kernel_stats.csv"
