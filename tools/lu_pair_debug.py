"""Debug helper (r05): factor one small matrix with the paired-block default and with IADMM_LU_RANK128
and report where the packed factors differ (by 64 x 64 region), to localise a fault in the paired
rank-256 update."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 384
g = torch.Generator().manual_seed(5)
K = (torch.randn(1, N, N, generator=g) + 4 * torch.eye(N)).cuda()  # diagonally heavy: few interchanges
out = {}
for fl in (ops.LU_RANK128, 0):
    LU, piv, info = ops.lu_factor(K.clone(), flags=fl, lookahead=False)
    torch.cuda.synchronize()
    out[fl] = (LU[0].cpu(), piv[0].cpu(), int(info[0]))
a, b = out[ops.LU_RANK128], out[0]
print("info", a[2], b[2], "piv equal", torch.equal(a[1], b[1]), "first piv diff", (a[1] != b[1]).nonzero()[:3].flatten().tolist())
d = (a[0] - b[0]).abs()
for r0 in range(0, N, 64):
    print(f"rows {r0:4d}: " + " ".join(f"{float(d[r0:r0 + 64, c0:c0 + 64].max()):8.1e}" for c0 in range(0, N, 64)))
print("paired sample row 300, cols 256..263:", b[0][300, 256:264].tolist())
print("rank128 sample row 300, cols 256..263:", a[0][300, 256:264].tolist())
