"""Debug (r05): factor the same KKT batch (tools/lu_ab.py's, B = 1024, N = 2000) with two library builds
(IADMM_LIB_PATH; child processes) -- and the second build twice -- and report which instances' factors
differ (per-instance bit sums), then the first differing entry of the first such instance with its
128-column block / 64-column half / 16-column panel.
    python tools/lu_ll_debug.py variants/lu_noll.so i-admm-lstm_amd/iadmm/libiadmm.so"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out, B, N, keep):
    sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
    import torch
    from iadmm import data, ops
    n = N // 2
    mi = me = n // 2
    d = data.make_qp_batch(n, mi, me, B, device="cuda")
    rho = torch.full((B, mi + me), 0.5, device="cuda")
    rho[:, mi:] = 500.0
    K = ops.kkt_assemble(d["Q"], d["A0"], 6e-6, None, 0, rho_rows=rho)
    del d
    LU, piv, info = ops.lu_factor(K)
    sums = torch.stack([torch.sum(LU[i].view(torch.int32), dtype=torch.int64) for i in range(B)]).cpu().numpy()
    np.savez(out, sums=sums, piv=piv.cpu().numpy(), LU=LU[keep].cpu().numpy() if keep >= 0 else np.zeros(1))


if __name__ == "__main__":
    if sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]))
        sys.exit(0)
    libs = [sys.argv[1], sys.argv[2], sys.argv[2]]
    B, N = 1024, 2000
    res = []
    for i, lib in enumerate(libs):
        out = f"/tmp/lu_dbg_{i}.npz"
        subprocess.run([sys.executable, __file__, "--child", out, str(B), str(N), "-1"], check=True,
                       env=dict(os.environ, IADMM_LIB_PATH=os.path.abspath(lib)))
        res.append(np.load(out))
    bad = np.nonzero(res[0]["sums"] != res[1]["sums"])[0]
    rep = np.nonzero(res[1]["sums"] != res[2]["sums"])[0]
    print(f"instances differing A vs B: {len(bad)} {bad[:20].tolist()}; B run-to-run: {len(rep)} {rep[:20].tolist()}")
    pbad = np.nonzero((res[0]["piv"] != res[1]["piv"]).any(1))[0]
    print(f"instances with differing pivots: {len(pbad)} {pbad[:20].tolist()}")
    if len(bad):
        k = int(bad[0])
        lus = []
        for i, lib in enumerate(libs[:2]):
            out = f"/tmp/lu_dbg_k{i}.npz"
            subprocess.run([sys.executable, __file__, "--child", out, str(B), str(N), str(k)], check=True,
                           env=dict(os.environ, IADMM_LIB_PATH=os.path.abspath(lib)))
            lus.append(np.load(out))
        a, c = lus[0]["LU"], lus[1]["LU"]
        d = np.argwhere(a.view(np.int32) != c.view(np.int32))
        r, col = d[np.lexsort((d[:, 0], d[:, 1]))][0]
        print(f"instance {k}: {len(d)} entries differ; first (by column) row {r} col {col} (block {col // 128}, half "
              f"{(col % 128) // 64}, panel {(col % 64) // 16}); values {a[r, col]} vs {c[r, col]}; "
              f"rows differing in that column: {np.nonzero(a[:, col].view(np.int32) != c[:, col].view(np.int32))[0][:20].tolist()}")
        pa, pc = lus[0]["piv"][k], lus[1]["piv"][k]
        dp = np.nonzero(pa != pc)[0]
        print(f"first differing pivot of instance {k}: {dp[:5].tolist()} {pa[dp[:5]].tolist()} vs {pc[dp[:5]].tolist()}")
