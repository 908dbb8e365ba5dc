#!/bin/bash
# r04 session 8: the default bench line at HEAD (as the driver runs it)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/r04g2_bench.log 2>&1 || exit $?
grep '^{' gpurun_out/r04g2_bench.log > gpurun_out/r04g2_bench.json
python3 - <<'PY'
import json
r = json.loads(open("gpurun_out/r04g2_bench.json").read().strip().splitlines()[-1])
print("value", r["value"], r["unit"], "ms/step", r["ms_per_step"])
print("roofline", {k: r["roofline"].get(k) for k in ("achieved", "frac", "traffic")})
s2 = r.get("stage2", {})
print("stage2", {k: s2.get(k) for k in ("factor_ms", "instances_per_s", "solve_ms")}, s2.get("roofline", {}).get("frac"), s2.get("roofline", {}).get("traffic"))
print("train", r.get("train", {}).get("roofline", {}).get("frac"))
print("resid", r.get("final_residual"))
PY
