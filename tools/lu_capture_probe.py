"""does capturing the LU's fork / join (rank-128 look-ahead, N > 2048) or its batch
split (paired form, B >= 512) into a hipGraph work?  Run against a variant build without the capture
guards (IADMM_LIB_PATH=tools/var_lu_capture.so): capture factor + solve on a side stream with
torch.cuda.graph, replay twice, compare bit for bit with eager runs.  Prints one JSON line per case."""
import faulthandler
import json
import os
import sys
import time

faulthandler.enable()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import ops, _abi  # noqa: E402


def case(N, B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    K = torch.randn(B, N, N, generator=g, device="cuda")
    K[:, 0, 0] = 0.0
    b = torch.randn(B, N, generator=g, device="cuda")
    LU0, piv0, info0 = ops.lu_factor(K.clone())
    x0 = ops.lu_solve(LU0, piv0, b)
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    Ks, bs = K.clone(), b.clone()
    ws = ops.lu_factor_ws(B, N, K.device)
    with torch.cuda.stream(s):
        ops.lu_factor(Ks.clone(), ws=ws)
    s.synchronize()
    print(f"[probe] N={N} B={B}: capturing", flush=True)
    t0 = time.time()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        A = Ks.clone()
        LU, piv, info = ops.lu_factor(A, ws=ws)
        x = ops.lu_solve(LU, piv, bs)
    print(f"[probe] N={N} B={B}: captured in {time.time() - t0:.2f} s", flush=True)
    same = []
    for _ in range(2):
        gr.replay()
        torch.cuda.synchronize()
        same.append(bool(torch.equal(LU, LU0) and torch.equal(piv, piv0) and torch.equal(x, x0)))
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    gr.replay()
    ev1.record()
    torch.cuda.synchronize()
    replay_ms = ev0.elapsed_time(ev1)
    ev0.record()
    LU2, piv2, _ = ops.lu_factor(K.clone(), ws=ws)
    ops.lu_solve(LU2, piv2, b)
    ev1.record()
    torch.cuda.synchronize()
    print(json.dumps(dict(lib=_abi.LIB_PATH, N=N, B=B, replay_bitwise=same, replay_ms=replay_ms,
                          eager_ms=ev0.elapsed_time(ev1))), flush=True)


if __name__ == "__main__":
    case(2500, 4, 12)       # rank-128 blocks: the look-ahead's fork / join on the context's streams
    case(2000, 512, 13)     # paired blocks: the batch split over the context's two streams
    case(2500, 256, 14)     # look-ahead at a batch that fills the chip
