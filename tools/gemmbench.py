"""Training-GEMM timing (iadmm_gemm_nt / iadmm_gemm_tn at the config-5 microbatch shape) over
library builds: python tools/gemmbench.py [extra .so ...].  Prints ms and TFLOP/s per call and the
max relative difference to the in-tree build."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import _abi  # noqa: E402


def bind(path):
    lib = ctypes.CDLL(path)
    for name in ("iadmm_gemm_nt", "iadmm_gemm_tn", "iadmm_gemm_tn_splits", "iadmm_gemm_pack_a",
                 "iadmm_gemm_packed_a_floats", "iadmm_gemm_nt_packed"):
        f = getattr(lib, name)
        f.restype, f.argtypes = _abi.SIGNATURES[name]
    return lib


def timeit(fn, iters=5):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    M, h = int(os.environ.get("GB_M", 256000)), int(os.environ.get("GB_H", 800))
    libs = [os.path.join(ROOT, "i-admm-lstm_amd", "iadmm", "libiadmm.so")] + sys.argv[1:]
    torch.manual_seed(0)
    H = torch.randn(M, h, device="cuda")
    dP = torch.randn(M, 4 * h, device="cuda")
    U = torch.randn(h, 4 * h, device="cuda")
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    flop = 2.0 * M * h * 4 * h
    ref_nt = ref_tn = None
    for path in libs:
        lib = bind(path)
        name = os.path.basename(path)
        out_nt = torch.empty(M, h, device="cuda")
        t_nt = timeit(lambda: lib.iadmm_gemm_nt(M, h, 4 * h, p(dP), p(U), p(out_nt), 0, st))
        Wpk = torch.empty(int(lib.iadmm_gemm_packed_a_floats(h, 4 * h)), device="cuda")
        lib.iadmm_gemm_pack_a(h, 4 * h, p(U), p(Wpk), st)
        out_pk = torch.empty(M, h, device="cuda")
        t_pk = timeit(lambda: lib.iadmm_gemm_nt_packed(M, h, 4 * h, p(dP), p(Wpk), p(out_pk), 0, st))
        d_pk = float((out_pk - out_nt).abs().max() / out_nt.abs().max())
        print(f"{name:20s} gemm_nt packed-A {t_pk:8.3f} ms {flop / t_pk / 1e9:7.1f} TF (vs row-major: diff {d_pk:.1e})",
              flush=True)
        rps = int(os.environ.get("GB_RPS", 4096))
        ns = lib.iadmm_gemm_tn_splits(M, rps)
        slab = torch.empty(ns, h, 4 * h, device="cuda")
        out_tn = torch.empty(h, 4 * h, device="cuda")
        t_tn = timeit(lambda: lib.iadmm_gemm_tn(M, h, 4 * h, rps, p(H), p(dP), p(slab), p(out_tn), 0, st))
        d_nt = 0.0 if ref_nt is None else float((out_nt - ref_nt).abs().max() / ref_nt.abs().max())
        d_tn = 0.0 if ref_tn is None else float((out_tn - ref_tn).abs().max() / ref_tn.abs().max())
        ref_nt = out_nt if ref_nt is None else ref_nt
        ref_tn = out_tn if ref_tn is None else ref_tn
        print(f"{name:20s} gemm_nt {t_nt:8.3f} ms {flop / t_nt / 1e9:7.1f} TF (diff {d_nt:.1e})   "
              f"gemm_tn {t_tn:8.3f} ms {flop / t_tn / 1e9:7.1f} TF (diff {d_tn:.1e})", flush=True)


if __name__ == "__main__":
    main()
