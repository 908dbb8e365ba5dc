#!/bin/bash
# r04 session 8: the default bench line at the final HEAD (as the driver runs it), after the K = 100
# parity tests with the final checkpoint
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh r04h2 600 tests/test_k100_gpu.py || exit $?
timeout -k 10 900 python -u bench.py > gpurun_out/r04h2_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r04h2_bench.log > gpurun_out/r04h2_bench.json
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r04h2_bench.json").read().strip().splitlines()[-1])
print("value", r["value"], r["unit"], "ms/step", r["ms_per_step"])
print("roofline", {k: r["roofline"].get(k) for k in ("achieved", "frac", "traffic")})
s2 = r.get("stage2", {})
print("stage2", {k: s2.get(k) for k in ("value", "factor_ms", "solve_iter_ms")}, s2.get("roofline", {}).get("frac"), s2.get("roofline", {}).get("frac_vs_box"), s2.get("roofline", {}).get("traffic"))
print("train", r.get("train", {}).get("roofline", {}).get("frac"))
print("resid", r.get("final_residual"))
PY
