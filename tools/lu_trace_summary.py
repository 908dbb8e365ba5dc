"""Summarise an LU kernel trace (tools/gpu_r05d.sh: iadmm kernels only): per kernel family the
launch count and summed duration, the wall span from the first to the last LU kernel, and for the
trailing updates every launch's duration with its A22 size (r05 paired-block study).
    python tools/lu_trace_summary.py gpurun_out/r05d/pair1_kernel_trace.csv [N]"""
import csv
import re
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rows = [r for r in rows if "kkt_assemble" not in r["Kernel_Name"]]
t0 = min(int(r["Start_Timestamp"]) for r in rows)
t1 = max(int(r["End_Timestamp"]) for r in rows)
fam = defaultdict(lambda: [0, 0.0])
for r in rows:
    name = re.sub(r"^void |\(.*$", "", r["Kernel_Name"]).replace("iadmm::", "")
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    fam[name][0] += 1
    fam[name][1] += d
print(f"wall {((t1 - t0) / 1e6):.2f} ms over {len(rows)} launches")
for k, (c, t) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
    print(f"  {k[:60]:60s} {c:5d} {t:8.2f} ms")
