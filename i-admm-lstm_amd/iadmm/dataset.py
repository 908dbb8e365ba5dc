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


def write_qp(dir_path, d, num_ineq, first_index=0, solutions=None, prob_type="QP"):
    """Write a batch from :func:`iadmm.data.make_qp_batch` (Q already doubled) as qp_{i}.gz files
    (generate_data.py:85-92 layout).  ``solutions`` = optional (x[B,n], y[B,m]) stored as 'x'/'y'."""
    os.makedirs(dir_path, exist_ok=True)
    host = {k: d[k].detach().double().cpu().numpy() for k in REQUIRED}
    B = host["Q"].shape[0]
    mi = num_ineq
    for i in range(B):
        A0 = host["A0"][i]
        zl, zu = host["zl"][i].reshape(-1, 1), host["zu"][i].reshape(-1, 1)
        rec = {"Q": 0.5 * host["Q"][i], "p": host["p"][i].reshape(-1, 1), "A0": A0, "zl": zl, "zu": zu}
        if mi > 0:
            rec.update(G=A0[:mi], c=zu[:mi])
        if A0.shape[0] > mi:
            rec.update(A=A0[mi:], b=zu[mi:])
        if solutions is not None:
            rec.update(x=solutions[0][i].detach().double().cpu().numpy().reshape(-1),
                       y=solutions[1][i].detach().double().cpu().numpy().reshape(-1))
        with gzip.open(instance_file(dir_path, first_index + i, prob_type), "wb") as f:
            pickle.dump(rec, f)


def read_qp(dir_path, ids, device, prob_type="QP", qplib_num=None):
    """Load instances ``ids`` (main.py:621-722).  Returns dict of float32 tensors on ``device``:
    Q[B,n,n] (doubled), p[B,n,1], A0[B,m,n], zl/zu[B,m,1], and G/c, A/b, lb/ub when present in
    every file.  Sparse (scipy) arrays of the non-QP types are densified like main.py:661-705.
    Raises FileNotFoundError naming the first missing file."""
    if len(ids) == 0:
        raise ValueError("no instance ids to load")
    cols = {}
    for i in ids:
        path = instance_file(dir_path, i, prob_type, qplib_num)
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        with gzip.open(path, "rb") as f:
            rec = pickle.load(f)  # trusted user dataset in the reference's format
        missing = [k for k in REQUIRED if k not in rec]
        if missing:
            raise KeyError(f"{path}: missing {missing}")
        for k, v in rec.items():
            if hasattr(v, "toarray"):
                v = v.toarray()
            cols.setdefault(k, []).append(np.asarray(v, dtype=np.float64))
    out = {}
    for k in REQUIRED + tuple(k for pair in OPTIONAL for k in pair):
        if k in cols and len(cols[k]) == len(ids):
            a = np.stack(cols[k])
            if k in ("p", "zl", "zu", "c", "b", "lb", "ub") and a.ndim == 2:
                a = a[..., None]
            out[k] = torch.tensor(a, dtype=torch.float32, device=device)
    out["Q"] = out["Q"] * 2
    return out
