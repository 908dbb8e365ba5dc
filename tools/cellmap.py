"""Cell-kernel tile-order study: time iadmm_lstm_cell_fwd at the bench shape (B instances of
n + m = 2000 rows, h = 800) for several IADMM_CELL_PGROUP values (cell_tile.h
cell_tile_of_block_grouped: row panels per group, hidden tile slowest inside a group).

  python tools/cellmap.py [--batch 1024] [--groups 1 2 3 4 5 8] [--reps 5]

Prints one JSON line per group size (mean ms per launch over hipEvents, TF/s against the fp32
MFMA spec) and checks that every order gives bitwise the same H', C' and projection partials.

r05: the product library no longer reads IADMM_CELL_PGROUP (include/iadmm.h: no environment reads;
the study's result, 4 panels per group, is built in).  Rerunning the study needs a variant build
(tools/build_variant.sh) with the getenv line restored in csrc/lstm.hip; the r02 results are in
profiles/r02_cellmap_*."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
import torch  # noqa: E402
from iadmm import data, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--rows", type=int, default=2000)
    ap.add_argument("--hidden", type=int, default=800)
    ap.add_argument("--groups", type=int, nargs="*", default=[1, 2, 3, 4, 5, 8])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    B, N, h = a.batch, a.rows, a.hidden
    params = data.init_lstm_params(h, 4, device="cuda")
    Upk, Wx = ops.lstm_pack(params, h)
    g = torch.Generator(device="cuda").manual_seed(3)
    H = torch.randn(B, N, h, device="cuda", generator=g) * 0.5
    C0 = torch.randn(B, N, h, device="cuda", generator=g) * 0.5
    C = C0.clone()
    Hn = torch.empty_like(H)
    xv, gg = torch.randn(B, N, device="cuda", generator=g), torch.randn(B, N, device="cuda", generator=g)
    part = torch.empty(ops.lstm_ntiles(h), B * N, device="cuda")
    flop = B * (8.0 * N * h * h + 18.0 * N * h)
    ref = None
    for pg in a.groups:
        os.environ["IADMM_CELL_PGROUP"] = str(pg)
        C.copy_(C0)
        ops.lstm_cell(H, C, xv, gg, Upk, Wx, Hn=Hn, Cn=C, part=part)
        torch.cuda.synchronize()
        got = (Hn.clone(), C.clone(), part.clone())
        if ref is None:
            ref = got
        same = all(torch.equal(x, y) for x, y in zip(got, ref))
        del got
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            ops.lstm_cell(H, C, xv, gg, Upk, Wx, Hn=Hn, Cn=C, part=part)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        print(json.dumps({"pgroup": pg, "ms": ms, "tflops": flop / ms / 1e9, "frac": flop / ms / 1e9 / 157.3,
                          "bitwise_equal_pgroup1": same}), flush=True)


if __name__ == "__main__":
    main()
