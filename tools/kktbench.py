"""Residual-matvec (iadmm_kkt_resgrad) bandwidth sweep over library builds and instance shapes.

  python tools/kktbench.py [extra .so paths ...]

Times 10 launches per (library, shape) with hipEvents on the current stream and prints the
algorithmic GB/s (2 reads of Q and A0 + the vectors); checks every library's g
against the in-tree build (max relative difference)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import _abi, ops  # noqa: E402


def load(path):
    lib = ctypes.CDLL(path)
    fn = lib.iadmm_kkt_resgrad
    fn.restype, fn.argtypes = _abi.SIGNATURES["iadmm_kkt_resgrad"]
    return fn


def run(fn, B, n, mi, me, iters=10):
    m = mi + me
    N = n + m
    torch.manual_seed(0)
    Q = torch.randn(B, n, n, device="cuda")
    A0 = torch.randn(B, m, n, device="cuda")
    p, x = torch.randn(B, n, device="cuda"), torch.randn(B, n, device="cuda")
    y, z = torch.randn(B, m, device="cuda"), torch.randn(B, m, device="cuda")
    xv = torch.randn(B, N, device="cuda")
    scal = ops.schedule(torch.zeros(4, 1, device="cuda"), torch.zeros(4, 1, device="cuda"), 0)
    g = torch.empty(B, N, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def call():
        rc = fn(B, n, m, mi, ptr(Q), ptr(A0), ptr(p), ptr(x), ptr(y), ptr(z), ptr(xv), 6e-6, ptr(scal), ptr(g),
                None, None, None, ctypes.c_void_p(st))
        assert rc == 0, rc

    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    byts = B * (2.0 * (n * n + m * n) * 4 + 10.0 * N * 4)
    out = g.clone()
    del Q, A0
    torch.cuda.empty_cache()
    return ms, byts / ms / 1e6, out


def main():
    libs = [os.path.join(ROOT, "i-admm-lstm_amd", "iadmm", "libiadmm.so")] + sys.argv[1:]
    fns = [(os.path.basename(p), load(p)) for p in libs]
    shapes = [(1024, 1000, 500, 500), (256, 2000, 1000, 1000), (128, 3000, 1500, 1500), (256, 5000, 2500, 2500)]
    for B, n, mi, me in shapes:
        ref = None
        for name, fn in fns:
            ms, gbs, g = run(fn, B, n, mi, me)
            diff = 0.0 if ref is None else float(((g - ref).abs().max() / ref.abs().max()))
            ref = g if ref is None else ref
            print(f"B={B:5d} n={n:5d} m={mi + me:5d} {name:22s} {ms:9.3f} ms  {gbs:8.1f} GB/s  maxdiff {diff:.2e}",
                  flush=True)


if __name__ == "__main__":
    main()
