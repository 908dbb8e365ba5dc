"""Co-residency phase study of the cell kernel from DIAG-6 stamps (tools/cellbench.bin B 1 phase
out.bin): per workgroup (start, main-loop end, operands landed, end, HW_ID, XCC_ID).  Groups the
workgroups by CU (XCC, SE, SH, CU fields of HW_ID), and reports over the steady part of the launch
how much of each CU's time had 0 / 1 / 2 workgroups in their main loop, and how often a
workgroup's epilogue overlapped its partner's epilogue.

  python tools/cellphase.py gpurun_out/phase.bin"""
import sys

import numpy as np


def main():
    st = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 8).astype(np.int64)
    t0, tml, tc, te, hw, xcc = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4], st[:, 5]
    cu = ((xcc & 0xF) << 16) | (((hw >> 13) & 0x7) << 8) | (((hw >> 12) & 1) << 4) | ((hw >> 8) & 0xF)
    ucu = np.unique(cu)
    print(f"{len(st)} workgroups on {len(ucu)} CUs; wg time median {np.median(te - t0):.0f} cyc, "
          f"main loop {np.median(tml - t0):.0f}, epilogue {np.median(te - tml):.0f}")
    tot = np.zeros(3)
    overlap_epi, epi_total = 0.0, 0.0
    for c in ucu:
        idx = np.where(cu == c)[0]
        s, m, e = t0[idx], tml[idx], te[idx]
        lo, hi = np.percentile(s, 5), np.percentile(e, 95)  # steady part of the launch
        ev = [(x, +1, 0) for x in s] + [(x, -1, 0) for x in m] + [(x, +1, 1) for x in m] + [(x, -1, 1) for x in e]
        ev.sort()
        n_ml, n_ep, last = 0, 0, None
        for t, d, kind in ev:
            if last is not None and lo <= last and t <= hi:
                dt = t - last
                tot[min(n_ml, 2)] += dt
                if n_ep >= 2:
                    overlap_epi += dt
                if n_ep >= 1:
                    epi_total += dt
            if kind == 0:
                n_ml += d
            else:
                n_ep += d
            last = t
    frac = tot / tot.sum()
    print(f"CU time with 0 / 1 / 2 workgroups in their main loop: {frac[0]:.3f} / {frac[1]:.3f} / {frac[2]:.3f}")
    print(f"time with >= 1 epilogue running: {epi_total / tot.sum():.3f}; with 2 epilogues at once: "
          f"{overlap_epi / tot.sum():.3f}")


if __name__ == "__main__":
    main()
