"""The reference's on-disk QP instance format: one gzip-pickled dict of dense float64 numpy arrays
per instance, ``<data_dir>/QP_{n}_{ineq}_{eq}/qp_{id}.gz``.

Writer side follows generate_data.py:85-92 (QP branch): keys Q (= 0.5 diag(u); the loader doubles
it), p [n,1], G [mi,n], c [mi,1], A [me,n], b [me,1], A0 = [G; A], zl = [-inf; b], zu = [c; b],
plus the solver's x / y when known.  Reader side follows main.py:621-722: Q, p, A0, zl, zu are
required; G/c, A/b and lb/ub are optional (KeyError -> that class is empty); every array becomes a
float32 device tensor and Q is doubled (main.py:718).

Only open datasets you trust: the format is pickle, which can execute code when loaded
(the reference's own choice of format; this module only restates it).
"""
from __future__ import annotations

import gzip
import os
import pickle
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

REQUIRED = ("Q", "p", "A0", "zl", "zu")
OPTIONAL = (("G", "c"), ("A", "b"), ("lb", "ub"))


# prob_type -> (dataset directory, per-instance file), main.py:78-165 and :621-650.  The solve path is
# the same for every type (models/lstm.py:47-96 uses only Q, p, A0, zl, zu); they differ in naming
# and in whether the arrays are stored dense (QP, QP_RHS) or as scipy sparse matrices.
LAYOUTS = {
    "QP": ("QP_{n}_{mi}_{me}", "qp_{i}.gz"),
    "QP_RHS": ("QP_RHS_{n}_{mi}_{me}", "qp_rhs_{i}.gz"),
    "Random_QP": ("Random_QP_{n}_{mi}", "random_qp_{i}.gz"),
    "Equality_QP": ("Equality_QP_{n}_{me}", "equality_qp_{i}.gz"),
    "SVM": ("SVM_{n}_{mi}", "svm_{i}.gz"),
    "QPLIB": ("QPLIB_{qplib}", "qplib_{qplib}_{i}.gz"),
    "MM_MOSARQP2": ("MM_MOSARQP2", "mosarqp2_{i}.gz"),
    "MM_QSCSD6": ("MM_QSCSD6", "qscsd6_{i}.gz"),
    "MM_QSCRS8": ("MM_QSCRS8", "qscrs8_{i}.gz"),
    "MM_Q25FV47": ("MM_Q25FV47", "q25fv47_{i}.gz"),
    "MM_QSHIP04L": ("MM_QSHIP04L", "qship04l_{i}.gz"),
    "MM_QSHIP08S": ("MM_QSHIP08S", "qship08s_{i}.gz"),
    "MM_CVXQP1_M": ("MM_CVXQP1_M", "cvxqp1_m_{i}.gz"),
    "MM_CVXQP3_M": ("MM_CVXQP3_M", "cvxqp3_m_{i}.gz"),
}


def _layout(prob_type):
    if prob_type not in LAYOUTS:
        raise ValueError(f"unknown prob_type {prob_type!r}; one of {sorted(LAYOUTS)}")
    return LAYOUTS[prob_type]


def instance_dir(data_dir, n, num_ineq, num_eq, prob_type="QP", qplib_num=None):
    return os.path.join(data_dir, _layout(prob_type)[0].format(n=n, mi=num_ineq, me=num_eq, qplib=qplib_num))


def instance_file(dir_path, i, prob_type="QP", qplib_num=None):
    return os.path.join(dir_path, _layout(prob_type)[1].format(i=i, qplib=qplib_num))


def write_qp(dir_path, d, num_ineq, first_index=0, solutions=None, prob_type="QP", workers=None,
             compresslevel=1):
    """Write a batch from :func:`iadmm.data.make_qp_batch` (Q already doubled) as qp_{i}.gz files
    (generate_data.py:85-92 layout).  ``solutions`` = optional (x[B,n], y[B,m]) stored as 'x'/'y'.
    Files are compressed on ``workers`` threads (zlib releases the GIL; default min(16, CPUs)) at
    ``compresslevel`` 1: the reference's gzip.open default (9) spends 21 s per n = 1000 instance
    on the mostly-zero diagonal Q (level 6: 2.5 s, level 1: 0.6 s for a 14 % larger file;
    tools/loaderbench.py).  Any level reads back identically."""
    os.makedirs(dir_path, exist_ok=True)
    host = {k: d[k].detach().double().cpu().numpy() for k in REQUIRED}
    sol = None if solutions is None else tuple(t.detach().double().cpu().numpy() for t in solutions)
    B = host["Q"].shape[0]
    mi = num_ineq

    def one(i):
        A0 = host["A0"][i]
        zl, zu = host["zl"][i].reshape(-1, 1), host["zu"][i].reshape(-1, 1)
        rec = {"Q": 0.5 * host["Q"][i], "p": host["p"][i].reshape(-1, 1), "A0": A0, "zl": zl, "zu": zu}
        if mi > 0:
            rec.update(G=A0[:mi], c=zu[:mi])
        if A0.shape[0] > mi:
            rec.update(A=A0[mi:], b=zu[mi:])
        if sol is not None:
            rec.update(x=sol[0][i].reshape(-1), y=sol[1][i].reshape(-1))
        with gzip.open(instance_file(dir_path, first_index + i, prob_type), "wb", compresslevel=compresslevel) as f:
            pickle.dump(rec, f, protocol=pickle.HIGHEST_PROTOCOL)

    _parallel(one, range(B), workers)


def _workers(workers):
    return max(1, int(workers) if workers else min(16, os.cpu_count() or 1))


def _parallel(fn, items, workers):
    """fn over items on a thread pool (in order of completion; exceptions re-raised)."""
    items = list(items)
    nw = _workers(workers)
    if nw == 1 or len(items) <= 1:
        for it in items:
            fn(it)
        return
    with ThreadPoolExecutor(max_workers=nw) as ex:
        for f in [ex.submit(fn, it) for it in items]:
            f.result()


def _gunzip(raw):
    """One-call inflate of a single-member gzip file (the GIL is released for the whole buffer;
    GzipFile.read inflates in small Python-level chunks); other files via gzip.decompress."""
    d = zlib.decompressobj(31)
    out = d.decompress(raw)
    if d.eof and not d.unused_data:
        return out
    return gzip.decompress(raw)


def _load_record(path):
    with open(path, "rb") as f:
        raw = f.read()
    rec = pickle.loads(_gunzip(raw))  # trusted user dataset in the reference's format
    missing = [k for k in REQUIRED if k not in rec]
    if missing:
        raise KeyError(f"{path}: missing {missing}")
    return rec


def _dense(v):
    return v.toarray() if hasattr(v, "toarray") else v


def read_qp(dir_path, ids, device, prob_type="QP", qplib_num=None, workers=None):
    """Load instances ``ids`` (main.py:621-722).  Returns dict of float32 tensors on ``device``:
    Q[B,n,n] (doubled), p[B,n,1], A0[B,m,n], zl/zu[B,m,1], and G/c, A/b, lb/ub when present in
    every file.  Sparse (scipy) arrays of the non-QP types are densified like main.py:661-705.
    Raises FileNotFoundError naming the first missing file.

    Files are decompressed on ``workers`` threads (default min(16, CPUs)) straight into one
    preallocated float32 array per key: the same fp64 -> fp32 rounding as the reference's
    ``torch.tensor(np.array(list), dtype=float32)``, without its float64 stack (1/4 of the host
    memory at the bench shape: 12 GB instead of ~48 GB for 1024 instances)."""
    if len(ids) == 0:
        raise ValueError("no instance ids to load")
    paths = [instance_file(dir_path, i, prob_type, qplib_num) for i in ids]
    for path in paths:
        if not os.path.exists(path):
            raise FileNotFoundError(path)
    keys = REQUIRED + tuple(k for pair in OPTIONAL for k in pair)
    first = _load_record(paths[0])
    shapes = {k: np.shape(_dense(first[k])) for k in keys if k in first}
    bufs = {k: np.empty((len(ids),) + shp, dtype=np.float32) for k, shp in shapes.items()}
    present = {k: np.zeros(len(ids), dtype=bool) for k in bufs}

    def fill(j, rec):
        for k, buf in bufs.items():
            if k in rec:
                v = np.asarray(_dense(rec[k]))
                if v.shape != shapes[k]:
                    raise ValueError(f"{paths[j]}: {k} has shape {v.shape}, instance {ids[0]} {shapes[k]}")
                buf[j] = v  # fp64 -> fp32, round to nearest (as torch.tensor(..., dtype=float32))
                present[k][j] = True

    fill(0, first)
    del first
    _parallel(lambda j: fill(j, _load_record(paths[j])), range(1, len(ids)), workers)
    out = {}
    for k in keys:
        if k in bufs and present[k].all():
            a = bufs[k]
            if k in ("p", "zl", "zu", "c", "b", "lb", "ub") and a.ndim == 2:
                a = a[..., None]
            out[k] = torch.from_numpy(a).to(device)
    out["Q"] = out["Q"] * 2
    return out
