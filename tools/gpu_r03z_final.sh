#!/bin/bash
# Round-end style run at HEAD: the whole -m gpu suite in one process, smoke(), the default bench line.
set -o pipefail
tag=${1:-r03zf}
mkdir -p gpurun_out/$tag
bash tools/gpu_suite.sh $tag || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$tag/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/$tag/smoke.log
timeout -k 10 900 python3 -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || exit 1
grep '^{' gpurun_out/$tag/bench.json | cut -c1-200
