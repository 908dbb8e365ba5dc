"""One batched LU factorization at a Stage-II shape (default config 2: B = 1024, N = 2000), for
rocprofv3 kernel-trace / PMC passes (tools/profile_lu.sh): the K assembly, one warm-up-free
factorization, nothing else on the GPU but the data generation."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=1024)
ap.add_argument("--N", type=int, default=2000)
ap.add_argument("--flags", type=int, default=0, help="iadmm_lu_factor_ex flags (4 = IADMM_LU_RANK128: the r04 form)")
ap.add_argument("--no-lookahead", action="store_true", help="every launch on one stream (clean durations)")
a = ap.parse_args()
from iadmm import data, ops  # noqa: E402
n = a.N // 2
mi = me = n // 2
d = data.make_qp_batch(n, mi, me, a.batch, device="cuda")
rho = torch.full((a.batch, mi + me), 0.5, device="cuda")
rho[:, mi:] = 500.0
K = ops.kkt_assemble(d["Q"], d["A0"], 6e-6, None, 0, rho_rows=rho)
del d
LU, piv, info = ops.lu_factor(K, flags=a.flags, lookahead=not a.no_lookahead)
torch.cuda.synchronize()
print(f"factored B={a.batch} N={a.N}: info max {int(info.max())}")
