"""ctypes binding of libiadmm.so (the C-ABI declared in include/iadmm.h).

Loading never touches the GPU, so the library can be loaded and its exports checked on a
machine without one.  A missing library raises immediately: there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(os.path.dirname(_HERE))


def _lib_path():
    """The in-tree product library.  IADMM_LIB_PATH names an alternative build of the same library for
    the variant studies of tools/ (tools/lu_ab.py, tools/cellbwd_ab.py, ...); it is honoured only for a
    .so under the repository's tools/ or variants/ directory, so the product path cannot be swapped
    for an arbitrary library."""
    own = os.path.join(_HERE, "libiadmm.so")
    alt = os.environ.get("IADMM_LIB_PATH")
    if not alt:
        return own
    real = os.path.realpath(alt)
    if real == os.path.realpath(own):
        return own
    roots = [os.path.realpath(os.path.join(_REPO, d)) + os.sep for d in ("tools", "variants")]
    if not real.endswith(".so") or not any(real.startswith(r) for r in roots):
        raise RuntimeError(f"IADMM_LIB_PATH={alt!r}: variant libraries must be .so files under tools/ or variants/")
    return real


LIB_PATH = _lib_path()

i64, f32, vp, cint = ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.c_int

# name -> (restype, argtypes); mirrors include/iadmm.h one for one.
SIGNATURES = {
    "iadmm_version": (cint, []),
    "iadmm_schedule": (cint, [vp, vp, i64, vp, vp]),
    "iadmm_schedule_fixed_alpha": (cint, [vp, f32, vp, vp]),
    "iadmm_kkt_resgrad_ws_bytes": (i64, [i64, i64, i64]),
    "iadmm_kkt_resgrad_lds_bytes": (i64, [i64, i64]),
    "iadmm_kkt_resgrad": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, i64,
                                 vp]),
    "iadmm_kkt_lsres": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp]),
    "iadmm_lstm_packed_floats": (i64, [i64]),
    "iadmm_lstm_wx_floats": (i64, [i64]),
    "iadmm_lstm_ntiles": (i64, [i64]),
    "iadmm_lstm_pack": (cint, [i64] + [vp] * 13 + [vp, vp, vp]),
    "iadmm_lstm_cell_fwd": (cint, [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_lstm_packed16_halfs": (i64, [i64]),
    "iadmm_lstm_pack_f16x3": (cint, [i64, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_split_f16": (cint, [i64, vp, vp, vp]),
    "iadmm_lstm_cell_fwd_f16x3": (cint, [i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_admm_update": (cint, [i64, i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, cint,
                                 vp, vp, vp, vp, vp, vp]),
    "iadmm_ruiz_scale": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_unscale": (cint, [i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_metrics": (cint, [i64, i64, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_bmv": (cint, [i64, i64, i64, vp, vp, vp, cint, vp, vp]),
    "iadmm_bmv_t": (cint, [i64, i64, i64, vp, vp, vp, vp]),
    "iadmm_bger": (cint, [i64, i64, i64, vp, vp, cint, vp, vp]),
    "iadmm_lu_factor_ws_bytes": (i64, [i64, i64]),
    "iadmm_lu_ctx_create": (cint, [ctypes.POINTER(vp)]),
    "iadmm_lu_ctx_destroy": (cint, [vp]),
    "iadmm_lu_factor": (cint, [i64, i64, vp, vp, vp, vp, i64, vp]),
    "iadmm_lu_factor_ex": (cint, [i64, i64, vp, vp, vp, vp, i64, vp, cint, vp]),
    "iadmm_lu_solve": (cint, [i64, i64, vp, vp, vp, vp]),
    "iadmm_lu_solve_ex": (cint, [i64, i64, vp, vp, vp, cint, vp]),
    "iadmm_kkt_assemble": (cint, [i64, i64, i64, i64, vp, vp, f32, vp, vp, vp, vp]),
    "iadmm_kkt_rhs": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, f32, vp, vp, vp, vp]),
    "iadmm_kkt_matvec": (cint, [i64, i64, i64, i64, vp, vp, vp, f32, vp, vp, cint, vp, vp]),
    "iadmm_gemm_nt": (cint, [i64, i64, i64, vp, vp, vp, cint, vp]),
    "iadmm_gemm_packed_a_floats": (i64, [i64, i64]),
    "iadmm_gemm_pack_a": (cint, [i64, i64, vp, vp, vp]),
    "iadmm_gemm_nt_packed": (cint, [i64, i64, i64, vp, vp, vp, cint, vp]),
    "iadmm_gemm_nt_kpart": (i64, [i64, i64]),
    "iadmm_gemm_nt_packed_split": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, cint, vp]),
    "iadmm_gemm_tn_splits": (i64, [i64, i64]),
    "iadmm_gemm_tn": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, cint, vp]),
    "iadmm_slab_reduce": (cint, [i64, i64, vp, vp, cint, vp]),
    "iadmm_admm_update_bwd": (cint, [i64, i64, i64, i64] + [vp] * 17 + [i64, vp]),
    "iadmm_lstm_cell_bwd": (cint, [i64, i64] + [vp] * 13 + [vp]),
    "iadmm_in_reduce": (cint, [i64, i64, vp, vp, vp, vp]),
    "iadmm_kkt_bwd": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp]),
    "iadmm_sched_bwd": (cint, [vp, vp, i64, vp, i64, vp, i64, vp, vp, vp, vp]),
    "iadmm_loss_grad": (cint, [i64, i64, i64] + [vp] * 13 + [vp]),
    "iadmm_kkt_bwd_split": (cint, [i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, f32, vp, vp, vp, vp, vp, vp, vp, i64,
                                   vp]),
    "iadmm_loss_grad_split": (cint, [i64, i64, i64] + [vp] * 14 + [i64, vp]),
    "iadmm_probe_mfma_flop": (i64, [i64, i64]),
    "iadmm_probe_mfma": (cint, [i64, i64, vp, vp]),
    "iadmm_probe_copy": (cint, [i64, vp, vp, vp]),
    "iadmm_probe_read": (cint, [i64, vp, vp, i64, i64, vp]),
}

ERRORS = {-1: "bad argument", -2: "size beyond kernel limit", -3: "misaligned pointer"}

_lib = None


class IadmmError(RuntimeError):
    pass


def lib():
    """The loaded library (loaded once).  Raises if it was not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: build it with `make -C i-admm-lstm_amd` or "
                "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def exported():
    """Names from SIGNATURES the library actually exports."""
    L = lib()
    return [n for n in SIGNATURES if getattr(L, n, None) is not None]


def call(name, *args):
    """Call an int-returning entry point; raise IadmmError on a non-zero status."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = ERRORS.get(rc, f"HIP error {rc}")
        raise IadmmError(f"{name} failed: {msg} (status {rc})")
    return rc
