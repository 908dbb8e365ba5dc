#!/bin/bash
# r03 session 2: default bench line (N=1) + rocprof kernel stats / PMC of the headline step.
set -o pipefail
tag=${1:-r03z}
mkdir -p gpurun_out/$tag
timeout -k 10 900 python3 -u bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || exit 1
grep '^{' gpurun_out/$tag/bench.json | cut -c1-300
bash tools/profile_bench.sh $tag || exit 1
echo done
