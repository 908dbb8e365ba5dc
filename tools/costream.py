"""Co-residency probe: does an HBM-streaming kernel run beside the cell kernel without taking its
CU slots?  (overlap of the residual matvec with the cell kernel.)

  python tools/costream.py            (needs tools/costream.so: hipcc --offload-arch=gfx950 -O3
                                        -shared -fPIC tools/costream.hip -o tools/costream.so)

Times, on one GPU: the cell kernel of B instances alone; a lean one-wave streaming reader alone;
the production residual matvec alone; and each reader launched on a second stream while the cell
kernel runs.  Prints one JSON line per case."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import data, ops  # noqa: E402


def ev():
    return torch.cuda.Event(enable_timing=True)


def main():
    lib = ctypes.CDLL(os.path.join(ROOT, "tools", "costream.so"))
    lib.costream_read.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]
    B, n, mi, me, h = 512, 1000, 500, 500, 800
    m, N = mi + me, 1000 + 1000
    params = data.init_lstm_params(h, 4, device="cuda")
    Upk, Wx = ops.lstm_pack(params, h)
    H = torch.randn(B, N, h, device="cuda") * 0.1
    C = torch.randn(B, N, h, device="cuda") * 0.1
    Hn = torch.empty_like(H)
    xv, g = torch.randn(B, N, device="cuda"), torch.randn(B, N, device="cuda")
    part = torch.empty(ops.lstm_ntiles(h), B * N, device="cuda")
    Bk = 512
    Q = torch.randn(Bk, n, n, device="cuda")
    A0 = torch.randn(Bk, m, n, device="cuda")
    p, x = torch.randn(Bk, n, device="cuda"), torch.randn(Bk, n, device="cuda")
    y, z = torch.randn(Bk, m, device="cuda"), torch.randn(Bk, m, device="cuda")
    xk = torch.randn(Bk, N, device="cuda")
    scal = ops.schedule(torch.zeros(4, 1, device="cuda"), torch.zeros(4, 1, device="cuda"), 0)
    gk = torch.empty(Bk, N, device="cuda")
    ws = ops.kkt_resgrad_ws(Bk, n, m, "cuda")
    kkt_bytes = Bk * 2.0 * (n * n + m * n) * 4
    big = torch.empty(int(kkt_bytes // 4), device="cuda").normal_()  # the bytes of one resgrad (2 passes)
    sink = torch.zeros(1 << 20, device="cuda")

    def cell():
        ops.lstm_cell(H, C, xv, g, Upk, Wx, Hn=Hn, Cn=C, part=part)

    def kkt():
        ops.kkt_resgrad(Q, A0, p, x, y, z, xk, 6e-6, scal, mi, g=gk, ws=ws)

    def lean(infl, chunk):
        def f():
            rc = lib.costream_read(big.data_ptr(), big.numel(), chunk, infl, sink.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream)
            assert rc == 0, rc
        return f

    def timed(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        a, b = ev(), ev()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps

    s2 = torch.cuda.Stream()
    t_cell = timed(cell)
    print(json.dumps({"case": "cell alone", "ms": t_cell}), flush=True)
    readers = {"kkt_resgrad": kkt}
    for infl in (2, 4, 6):
        for chunk in (1 << 16, 1 << 18):
            readers[f"lean infl={infl} chunk={chunk}"] = lean(infl, chunk)
    for name, fn in readers.items():
        t_alone = timed(fn)
        # concurrent: the cell kernel on the main stream, the reader on s2 started right after it
        torch.cuda.synchronize()
        a, b, c, d = ev(), ev(), ev(), ev()
        a.record()
        cell()
        b.record()
        with torch.cuda.stream(s2):
            c.record()
            fn()
            d.record()
        torch.cuda.synchronize()
        print(json.dumps({"case": name, "alone_ms": t_alone, "alone_GBs": kkt_bytes / t_alone / 1e6,
                          "with_cell: cell_ms": a.elapsed_time(b), "reader_ms": c.elapsed_time(d),
                          "reader_GBs": kkt_bytes / c.elapsed_time(d) / 1e6,
                          "cell_slowdown": a.elapsed_time(b) / t_cell - 1}), flush=True)


if __name__ == "__main__":
    main()
