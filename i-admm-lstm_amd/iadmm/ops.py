"""Tensor-level wrappers around the C-ABI (one function per kernel family).

Every wrapper takes contiguous fp32 tensors on the current HIP device, allocates its outputs
with the PyTorch caching allocator, launches on the current stream and returns.  There is no
host synchronisation and no CPU path: a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import ctypes
import threading

import torch

from . import _abi

NSCAL = 8  # IADMM_NSCAL
S_RHO_IN, S_RHO_EQ, S_IRHO_IN, S_IRHO_EQ, S_ALPHA, S_1MALPHA = range(6)


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _p(t):
    """Device pointer of a contiguous fp32 device tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("iadmm kernels need device tensors (no CPU fallback)")
    if t.dtype != torch.float32:
        raise TypeError(f"iadmm kernels compute in fp32, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError("iadmm kernels need contiguous tensors")
    return t.data_ptr()


def _c(t):
    return None if t is None else t.detach().float().contiguous()


def empty(*shape, like):
    return torch.empty(*shape, dtype=torch.float32, device=like.device)


# --------------------------------------------------------------------------- schedule
def schedule(rho_param, alpha_param, t, out=None):
    """Iteration scalars of step t (models/lstm.py:60-63) into a device [8] buffer."""
    out = empty(NSCAL, like=rho_param) if out is None else out
    _abi.call("iadmm_schedule", _p(rho_param), _p(alpha_param), int(t), _p(out), _stream())
    return out


def schedule_fixed_alpha(scal, alpha, out=None):
    out = torch.empty_like(scal) if out is None else out
    _abi.call("iadmm_schedule_fixed_alpha", _p(scal), float(alpha), _p(out), _stream())
    return out


# --------------------------------------------------------------------------- KKT
def kkt_resgrad_ws(B, n, m, device):
    """Workspace of iadmm_kkt_resgrad (row-dot, per-block partial and r vectors), reusable across
    calls of the same (B, n, m)."""
    nbytes = int(_abi.lib().iadmm_kkt_resgrad_ws_bytes(int(B), int(n), int(m)))
    return torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=device)


def kkt_resgrad(Q, A0, p, x, y, z, xv, sigma, scal, num_ineq, g=None, btild=None, rho_vec=None,
                r_out=None, ws=None):
    """g = K^T (K xv - b~) with the implicit KKT matrix (models/lstm.py:67-72).  ``ws``: a
    :func:`kkt_resgrad_ws` buffer (allocated per call when omitted)."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    g = empty(B, n + m, like=Q) if g is None else g
    ws = kkt_resgrad_ws(B, n, m, Q.device) if ws is None else ws
    _abi.call("iadmm_kkt_resgrad", B, n, m, int(num_ineq), _p(Q), _p(A0), _p(p), _p(x), _p(y), _p(z),
              _p(xv), float(sigma), _p(scal), _p(g), _p(btild), _p(rho_vec), _p(r_out), _p(ws),
              ws.numel() * 4, _stream())
    return g


def kkt_lsres(Q, A0, p, x, y, z, xv, sigma, scal, num_ineq, out=None):
    """Per-instance ||K xv - b~||_2 (main.py:952)."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    out = empty(B, like=Q) if out is None else out
    _abi.call("iadmm_kkt_lsres", B, n, m, int(num_ineq), _p(Q), _p(A0), _p(p), _p(x), _p(y), _p(z),
              _p(xv), float(sigma), _p(scal), _p(out), _stream())
    return out


# --------------------------------------------------------------------------- LSTM cell
def lstm_ntiles(h):
    return int(_abi.lib().iadmm_lstm_ntiles(int(h)))


def lstm_pack(params, h):
    """Pack W_*, U_*, b_*, W_h (models/lstm.py:21-38) into the cell kernel's layout."""
    L = _abi.lib()
    ref = params["U_i"]
    Upk = empty(int(L.iadmm_lstm_packed_floats(h)), like=ref)
    Wx = empty(int(L.iadmm_lstm_wx_floats(h)), like=ref)
    ps = [_c(params[k]) for k in ("W_i", "U_i", "b_i", "W_f", "U_f", "b_f", "W_o", "U_o", "b_o",
                                  "W_u", "U_u", "b_u", "W_h")]
    _abi.call("iadmm_lstm_pack", int(h), *[_p(t) for t in ps], _p(Upk), _p(Wx), _stream())
    return Upk, Wx


def lstm_cell(H, C, xv, g, Upk, Wx, Hn=None, Cn=None, part=None):
    """Fused LSTM cell over M rows; returns (Hn, Cn, part[ntiles, M]).  Cn may alias C."""
    h = H.shape[-1]
    M = H.numel() // h
    Hn = torch.empty_like(H) if Hn is None else Hn
    Cn = torch.empty_like(C) if Cn is None else Cn
    part = empty(lstm_ntiles(h), M, like=H) if part is None else part
    _abi.call("iadmm_lstm_cell_fwd", M, h, _p(H), _p(C), _p(xv), _p(g), _p(Upk), _p(Wx), _p(Hn), _p(Cn),
              _p(part), _stream())
    return Hn, Cn, part


# --------------------------------------------------------------------------- optional f16x3 cell
def _p16(t):
    """Device pointer of a contiguous fp16 device tensor (the split planes of csrc/lstm_f16x3.hip)."""
    if t is None:
        return None
    if not t.is_cuda or t.dtype != torch.float16 or not t.is_contiguous():
        raise TypeError("split planes must be contiguous float16 device tensors")
    return t.data_ptr()


def lstm_pack_f16x3(params, h):
    """Split, power-of-two-scaled gate weights (Upk16 [2 planes], wscale [2])."""
    L = _abi.lib()
    ref = params["U_i"]
    Upk16 = torch.empty(int(L.iadmm_lstm_packed16_halfs(h)), dtype=torch.float16, device=ref.device)
    wscale = empty(2, like=ref)
    us = [_c(params[k]) for k in ("U_i", "U_f", "U_o", "U_u")]
    _abi.call("iadmm_lstm_pack_f16x3", int(h), *[_p(t) for t in us], _p16(Upk16), _p(wscale), _stream())
    return Upk16, wscale


def split_f16(X, out=None):
    """[2, *X.shape] fp16 planes (hi, lo) of an fp32 tensor."""
    out = torch.empty((2,) + tuple(X.shape), dtype=torch.float16, device=X.device) if out is None else out
    _abi.call("iadmm_split_f16", X.numel(), _p(X), _p16(out), _stream())
    return out


def lstm_cell_f16x3(H16, C, xv, g, Upk16, wscale, Wx, Hn16=None, Cn=None, part=None, Hn=None):
    """Split-precision cell: H16 [2, M, h] planes -> (Hn16, Cn, part, Hn); Hn (fp32) only if given."""
    h = H16.shape[-1]
    M = H16[0].numel() // h
    Hn16 = torch.empty_like(H16) if Hn16 is None else Hn16
    Cn = torch.empty_like(C) if Cn is None else Cn
    part = empty(lstm_ntiles(h), M, like=C) if part is None else part
    _abi.call("iadmm_lstm_cell_fwd_f16x3", M, h, _p16(H16), _p(C), _p(xv), _p(g), _p16(Upk16), _p(Wx),
              _p(wscale), _p(Hn), _p16(Hn16), _p(Cn), _p(part), _stream())
    return Hn16, Cn, part, Hn


# --------------------------------------------------------------------------- ADMM update
def admm_update(n, m, num_ineq, part, b_h, xv, x, y, z, zl, zu, scal, relax_z=False, out=None,
                rho_vec=None, rho_rows=None):
    """xv' / x' / z' / y' (models/lstm.py:80-94; relax_z -> models/lu.py:38-45)."""
    B = x.shape[0]
    if out is None:
        out = (torch.empty_like(xv), torch.empty_like(x), torch.empty_like(y), torch.empty_like(z))
    xvo, xo, yo, zo = out
    ntiles = 0 if part is None else part.shape[0]
    _abi.call("iadmm_admm_update", B, n, m, int(num_ineq), ntiles, _p(part), _p(b_h), _p(xv), _p(x), _p(y),
              _p(z), _p(zl), _p(zu), _p(scal), _p(rho_rows), int(bool(relax_z)), _p(xvo), _p(xo), _p(yo), _p(zo),
              _p(rho_vec), _stream())
    return xvo, xo, yo, zo


# --------------------------------------------------------------------------- Ruiz / unscale / metrics
def ruiz_scale(Q, p, A0, zl, zu, iters=10, out=None):
    """Modified Ruiz + cost scaling (methods/scaling.py:50-119).  Returns
    (Q, p, A0, zl, zu, D[B,n], E[B,m], c[B]).  ``out`` may be the inputs (in place)."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    if out is None:
        out = (torch.empty_like(Q), torch.empty_like(p), torch.empty_like(A0), torch.empty_like(zl),
               torch.empty_like(zu))
    Qo, po, Ao, zlo, zuo = out
    D, E, c = empty(B, n, like=Q), empty(B, m, like=Q), empty(B, like=Q)
    _abi.call("iadmm_ruiz_scale", B, n, m, int(iters), _p(Q), _p(p), _p(A0), _p(zl), _p(zu), _p(Qo), _p(po),
              _p(Ao), _p(zlo), _p(zuo), _p(D), _p(E), _p(c), _stream())
    return Qo, po, Ao, zlo, zuo, D, E, c


def unscale(D, E, c, x, y, z, out=None):
    """x = D x, y = (c^-1 E) y, z = E^-1 z (main.py:1025-1027)."""
    B, n = x.shape[0], x.shape[1]
    m = y.shape[1]
    if out is None:
        out = (torch.empty_like(x), torch.empty_like(y), torch.empty_like(z))
    xo, yo, zo = out
    _abi.call("iadmm_unscale", B, n, m, _p(D), _p(E), _p(c), _p(x), _p(y), _p(z), _p(xo), _p(yo), _p(zo),
              _stream())
    return xo, yo, zo


def metrics(Q, p, A0, x, y, z):
    """(obj, primal, dual) per instance, each [B] (utils.py:53-54, 68-71)."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    obj, pr, du = empty(B, like=Q), empty(B, like=Q), empty(B, like=Q)
    _abi.call("iadmm_metrics", B, n, m, _p(Q), _p(p), _p(A0), _p(x), _p(y), _p(z), _p(obj), _p(pr), _p(du),
              _stream())
    return obj, pr, du


BMV_PLAIN, BMV_POS_EXCESS, BMV_ABS_GAP = 0, 1, 2


def bmv(Mx, x, rhs=None, mode=BMV_PLAIN):
    """Batched matvec with a fused metric epilogue: Mx x, clamp(Mx x - rhs, 0) or |rhs - Mx x|."""
    B, R, C = Mx.shape
    out = empty(B, R, like=Mx)
    _abi.call("iadmm_bmv", B, R, C, _p(Mx), _p(x), _p(rhs), int(mode), _p(out), _stream())
    return out


def bmv_t(Mx, v, out=None):
    """Batched transposed matvec Mx^T v: Mx [B,R,C], v [B,R] -> [B,C]."""
    B, R, C = Mx.shape
    out = empty(B, C, like=Mx) if out is None else out
    _abi.call("iadmm_bmv_t", B, R, C, _p(Mx), _p(v), _p(out), _stream())
    return out


def bger(u, v, out=None, accumulate=False):
    """Per-instance rank-1 product u v^T: u [B,R], v [B,C] -> [B,R,C] (added to ``out`` with
    ``accumulate``)."""
    B, R = u.shape
    C = v.shape[1]
    out = empty(B, R, C, like=u) if out is None else out
    _abi.call("iadmm_bger", B, R, C, _p(u), _p(v), int(bool(accumulate)), _p(out), _stream())
    return out


def kkt_matvec(Q, A0, v, sigma, scal, num_ineq, transpose=False, rho_rows=None):
    """Implicit K v or K^T v, v[B,n+m] -> [B,n+m]."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    out = empty(B, n + m, like=Q)
    _abi.call("iadmm_kkt_matvec", B, n, m, int(num_ineq), _p(Q), _p(A0), _p(v), float(sigma), _p(scal),
              _p(rho_rows), int(bool(transpose)), _p(out), _stream())
    return out


def kkt_assemble(Q, A0, sigma, scal, num_ineq, rho_rows=None):
    """Dense K[B,n+m,n+m] (rho per class from ``scal`` or per row from ``rho_rows`` [B,m])."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    K = empty(B, n + m, n + m, like=Q)
    _abi.call("iadmm_kkt_assemble", B, n, m, int(num_ineq), _p(Q), _p(A0), float(sigma), _p(scal),
              _p(rho_rows), _p(K), _stream())
    return K


def kkt_rhs(p, x, y, z, sigma, scal=None, num_ineq=0, rho_rows=None, out=None):
    """b~ = [sigma x - p ; z - y / rho], [B,n+m] (models/lu.py:30)."""
    B, n = x.shape[0], x.shape[1]
    m = y.shape[1]
    out = empty(B, n + m, like=x) if out is None else out
    _abi.call("iadmm_kkt_rhs", B, n, m, int(num_ineq), _p(p), _p(x), _p(y), _p(z), float(sigma), _p(scal),
              _p(rho_rows), _p(out), _stream())
    return out


def lu_factor_ws(B, N, device):
    """Workspace of iadmm_lu_factor (caller-owned, from the PyTorch caching allocator)."""
    nbytes = int(_abi.lib().iadmm_lu_factor_ws_bytes(int(B), int(N)))
    return torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=device)


LU_FORCE_HBM = 1  # include/iadmm.h IADMM_LU_FORCE_HBM (tests)
LU_PAIRS = 2      # include/iadmm.h IADMM_LU_PAIRS (rank-256 paired-block updates: the default since r05)
LU_RANK128 = 4    # include/iadmm.h IADMM_LU_RANK128 (the r04 rank-128 blocks with the look-ahead: A/B and tests)


class LuContext:
    """An iadmm_lu_ctx: the look-ahead's two priority streams and four events, owned by the caller
    (include/iadmm.h).  Made on the current device; destroyed with the object."""

    def __init__(self):
        h = ctypes.c_void_p()
        _abi.call("iadmm_lu_ctx_create", ctypes.byref(h))
        self.handle = h.value
        self.device = torch.cuda.current_device()

    def __del__(self):
        h, self.handle = getattr(self, "handle", None), None
        if h and _abi is not None:
            try:
                _abi.lib().iadmm_lu_ctx_destroy(h)
            except Exception:  # interpreter teardown
                pass


_LU_CTX = threading.local()  # per thread: OrderedDict (device, caller stream) -> LuContext
LU_CTX_PER_THREAD = 8        # least recently used contexts beyond this are destroyed


def lu_context():
    """The LuContext of the current (device, stream, thread): a context serves one factorization at a
    time in its streams' order, so concurrent callers -- other threads, other streams, a graph capture
    beside eager work -- each get their own.  Held in thread-local storage (a finished thread's
    contexts are destroyed with it) and at most LU_CTX_PER_THREAD per thread, least recently used
    evicted (a caller on fresh streams no longer leaks HIP streams and events; destroying
    a context waits for its streams' work, iadmm_lu_ctx_destroy)."""
    import collections
    cache = getattr(_LU_CTX, "map", None)
    if cache is None:
        cache = _LU_CTX.map = collections.OrderedDict()
    key = (torch.cuda.current_device(), torch.cuda.current_stream().cuda_stream)
    ctx = cache.get(key)
    if ctx is None:
        ctx = cache[key] = LuContext()
        while len(cache) > LU_CTX_PER_THREAD:
            cache.popitem(last=False)
    else:
        cache.move_to_end(key)
    return ctx


def lu_factor(K, ws=None, lookahead=True, flags=0):
    """In-place batched LU with partial pivoting: returns (LU (= K), piv int32 [B,N] 1-based (LAPACK), info int32 [B]).
    ``ws``: a :func:`lu_factor_ws` buffer (allocated per call when omitted).  ``lookahead``: factor the
    next block beside each trailing update on this caller's :func:`lu_context` (rank-128 blocks: N > 2048
    or :data:`LU_RANK128`; the factors are bit for bit the same either way).  ``flags``: 0,
    :data:`LU_FORCE_HBM`, :data:`LU_RANK128` (tests / A/B); :data:`LU_PAIRS` is the default."""
    if K.dim() != 3 or K.shape[1] != K.shape[2]:
        raise ValueError(f"K must be [B,N,N], got {tuple(K.shape)}")
    B, N = K.shape[0], K.shape[1]
    piv = torch.empty(B, N, dtype=torch.int32, device=K.device)
    info = torch.empty(B, dtype=torch.int32, device=K.device)
    ws = lu_factor_ws(B, N, K.device) if ws is None else ws
    ctx = lu_context().handle if lookahead else None
    _abi.call("iadmm_lu_factor_ex", B, N, _p(K), piv.data_ptr(), info.data_ptr(), _p(ws), ws.numel() * 4, ctx,
              int(flags), _stream())
    return K, piv, info


def lu_solve(LU, piv, b, flags=0):
    """Solve with (LU, piv) in place on a copy of b [B,N]; returns x.  ``flags``: 0 or :data:`LU_FORCE_HBM`."""
    B, N = LU.shape[0], LU.shape[1]
    if LU.dim() != 3 or LU.shape[2] != N:
        raise ValueError(f"LU must be [B,N,N], got {tuple(LU.shape)}")
    if piv.dtype != torch.int32 or not piv.is_contiguous():
        raise TypeError("piv must be contiguous int32")
    if not piv.is_cuda or piv.device != LU.device:
        raise ValueError("piv must be on the device of LU")
    if tuple(piv.shape) != (B, N) or b.numel() != B * N:
        raise ValueError(f"piv must be [B,N] = [{B},{N}] and b hold B*N values; got piv {tuple(piv.shape)}, "
                         f"b {tuple(b.shape)}")
    x = b.clone().contiguous()
    _abi.call("iadmm_lu_solve_ex", B, N, _p(LU), piv.data_ptr(), _p(x), int(flags), _stream())
    return x


# --------------------------------------------------------------------------- training backward
def gemm_nt(X, W, out=None, accumulate=False):
    """out[M,Ni] (+)= X[M,K] W[Ni,K]^T."""
    M, K = X.shape
    Ni = W.shape[0]
    out = empty(M, Ni, like=X) if out is None else out
    _abi.call("iadmm_gemm_nt", M, Ni, K, _p(X), _p(W), _p(out), int(bool(accumulate)), _stream())
    return out


def gemm_pack_a(W):
    """W[Ni,K] -> the packed tile layout of gemm_nt_packed."""
    Ni, K = W.shape
    Wpk = empty(int(_abi.lib().iadmm_gemm_packed_a_floats(Ni, K)), like=W)
    _abi.call("iadmm_gemm_pack_a", Ni, K, _p(W), _p(Wpk), _stream())
    return Wpk


def _cu_count():
    dev = torch.cuda.current_device()
    n = _CU_COUNT.get(dev)
    if n is None:
        n = _CU_COUNT[dev] = int(torch.cuda.get_device_properties(dev).multi_processor_count)
    return n


_CU_COUNT = {}
GEMM_FILL = 2  # workgroup slots per CU the small-M GEMM splits aim to fill (two 4-wave workgroups per CU)


def _gemm_tile(Ni):
    """csrc/gemm.hip gemm_nt_tile: 160-row output tiles when they pad Ni less than 128-row tiles."""
    w128, w160 = -(-Ni // 128) * 128 - Ni, -(-Ni // 160) * 160 - Ni
    return 160 if w160 < w128 else 128


def gemm_nt_ksplit(M, Ni, K):
    """K splits for gemm_nt_packed (r06): 1 while the output tiles alone fill GEMM_FILL workgroups per
    CU; below that (the recipe's batch 2: M = 4000, 80 tiles) as many splits of >= 256 K as fit in one
    round of those slots (6 of 544: 480 workgroups; 7 made 560 for 512 slots, a second round)."""
    tiles = -(-Ni // _gemm_tile(Ni)) * -(-M // 256)
    want = GEMM_FILL * _cu_count()
    if K % 16 or tiles >= want:
        return 1
    ks = min(want // tiles, max(1, K // 256))  # one round of workgroups (560 of 512 slots ran two)
    if ks <= 1:
        return 1
    kpart = int(_abi.lib().iadmm_gemm_nt_kpart(K, ks))
    return -(-K // kpart)


def gemm_nt_packed(X, Wpk, Ni, out=None, accumulate=False, ksplit=None):
    """out[M,Ni] (+)= X[M,K] W[Ni,K]^T with W pre-packed by gemm_pack_a.  ``ksplit``: K splits summed in
    split order (default gemm_nt_ksplit: 1 unless the output tiles leave CUs idle)."""
    M, K = X.shape
    out = empty(M, Ni, like=X) if out is None else out
    ks = gemm_nt_ksplit(M, Ni, K) if ksplit is None else int(ksplit)
    if ks <= 1:
        _abi.call("iadmm_gemm_nt_packed", M, Ni, K, _p(X), _p(Wpk), _p(out), int(bool(accumulate)), _stream())
        return out
    slab = empty(ks, M, Ni, like=X)
    _abi.call("iadmm_gemm_nt_packed_split", M, Ni, K, ks, _p(X), _p(Wpk), _p(slab), _p(out), int(bool(accumulate)),
              _stream())
    return out


def gemm_tn_rows_per_split(M, Ni, No, cap=4096):
    """Row slices for gemm_tn (r06): ``cap`` rows (the r01-r05 default: 4096 on MFMA, 512 for the
    skinny Ni <= 4 kernel) while the output tiles x slices fill GEMM_FILL workgroups per CU; fewer rows
    per slice (>= 256 / 32, a multiple of 32) when they do not (the recipe's batch 2: M = 4000 rows,
    65 output tiles -> 7 slices of 576 rows instead of 1 (one round of workgroups); the skinny d[W;b] GEMM 125 slices of 32
    rows instead of 8 of 512)."""
    if Ni <= 4:  # the streaming skinny kernel: 1024 columns x one slice per workgroup, 512-row slices
        tiles, cap, floor = -(-No // 1024), 512, 32
    else:
        tiles, floor = -(-Ni // _gemm_tile(Ni)) * -(-No // 256), 256
    ns = max(1, GEMM_FILL * _cu_count() // tiles)  # one round of workgroups
    rps = -(-M // ns)
    return int(min(cap, max(floor, -(-rps // 32) * 32)))


def gemm_tn(X, Y, rows_per_split=None, out=None, accumulate=False):
    """out[Ni,No] (+)= X[M,Ni]^T Y[M,No] (split over M, fixed-order reduction).  ``rows_per_split``:
    default gemm_tn_rows_per_split."""
    M, Ni = X.shape
    No = Y.shape[1]
    if rows_per_split is None:
        rows_per_split = gemm_tn_rows_per_split(M, Ni, No)
    ns = int(_abi.lib().iadmm_gemm_tn_splits(M, rows_per_split))
    slab = empty(ns, Ni, No, like=X)
    out = empty(Ni, No, like=X) if out is None else out
    _abi.call("iadmm_gemm_tn", M, Ni, No, rows_per_split, _p(X), _p(Y), _p(slab), _p(out),
              int(bool(accumulate)), _stream())
    return out


def slab_reduce(slab, out=None, accumulate=False):
    ns = slab.shape[0]
    nelem = slab[0].numel()
    out = empty(*slab.shape[1:], like=slab) if out is None else out
    _abi.call("iadmm_slab_reduce", nelem, ns, _p(slab), _p(out), int(bool(accumulate)), _stream())
    return out


UPD_BWD_BLOCKS = 256


def admm_update_bwd(n, m, num_ineq, x, y, z, xv_out, zl, zu, scal, dx_o, dy_o, dz_o, dxv_o):
    B = x.shape[0]
    dx, dy, dz = torch.empty_like(x), torch.empty_like(y), torch.empty_like(z)
    dxv, dq = torch.empty_like(xv_out), torch.empty_like(xv_out)
    partials = empty(UPD_BWD_BLOCKS, 4, like=x)
    _abi.call("iadmm_admm_update_bwd", B, n, m, int(num_ineq), _p(x), _p(y), _p(z), _p(xv_out), _p(zl), _p(zu),
              _p(scal), _p(dx_o), _p(dy_o), _p(dz_o), _p(dxv_o), _p(dx), _p(dy), _p(dz), _p(dxv), _p(dq),
              _p(partials), UPD_BWD_BLOCKS, _stream())
    return dx, dy, dz, dxv, dq, partials


def lstm_cell_bwd(H, C, xv, g, Upk, Wx, dq, dHn=None, dCn=None):
    h = H.shape[-1]
    M = H.numel() // h
    nrt, ntl = (M + 255) // 256, lstm_ntiles(h)
    dC = torch.empty_like(C)
    dP = empty(M, 4 * h, like=H)
    whslab = empty(nrt, h, like=H)
    inpart = empty(ntl, M, 2, like=H)
    _abi.call("iadmm_lstm_cell_bwd", M, h, _p(H), _p(C), _p(xv), _p(g), _p(Upk), _p(Wx), _p(dq), _p(dHn), _p(dCn),
              _p(dC), _p(dP), _p(whslab), _p(inpart), _stream())
    return dC, dP, whslab, inpart


def in_reduce(inpart, dxv, dg=None):
    ntl, M = inpart.shape[0], inpart.shape[1]
    dg = empty(M, like=inpart) if dg is None else dg
    _abi.call("iadmm_in_reduce", M, ntl, _p(inpart), _p(dxv), _p(dg), _stream())
    return dg


def kkt_bwd(Q, A0, xv, y, r, dg, sigma, scal, num_ineq, dxv, dx, dy, dz, split=True, ws=None):
    """Backward of :func:`kkt_resgrad` (accumulates into dxv, dx, dy, dz; returns ds per
    instance).  ``split``: the row-block split (iadmm_kkt_bwd_split, fills the chip at the
    training micro-batch); False: one workgroup per instance (iadmm_kkt_bwd)."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    ds = empty(B, like=Q)
    if split:
        ws = kkt_resgrad_ws(B, n, m, Q.device) if ws is None else ws
        _abi.call("iadmm_kkt_bwd_split", B, n, m, int(num_ineq), _p(Q), _p(A0), _p(xv), _p(y), _p(r), _p(dg),
                  float(sigma), _p(scal), _p(dxv), _p(dx), _p(dy), _p(dz), _p(ds), _p(ws), ws.numel() * 4,
                  _stream())
    else:
        _abi.call("iadmm_kkt_bwd", B, n, m, int(num_ineq), _p(Q), _p(A0), _p(xv), _p(y), _p(r), _p(dg),
                  float(sigma), _p(scal), _p(dxv), _p(dx), _p(dy), _p(dz), _p(ds), _stream())
    return ds


def sched_bwd(rho_param, alpha_param, t, upd_partials, kkt_ds, drho, dalpha, dbh):
    _abi.call("iadmm_sched_bwd", _p(rho_param), _p(alpha_param), int(t), _p(upd_partials), upd_partials.shape[0],
              _p(kkt_ds), kkt_ds.shape[0], _p(drho), _p(dalpha), _p(dbh), _stream())


def loss_grad(Q, p, A0, x, y, z, cp=None, cd=None, want_grad=True, split=True, ws=None):
    """(primal[B], dual[B], dx, dy, dz) of utils.py:68-71 with upstream coefficients cp, cd [B].
    ``split`` as for :func:`kkt_bwd` (iadmm_loss_grad_split / iadmm_loss_grad)."""
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    pr, du = empty(B, like=Q), empty(B, like=Q)
    dx = dy = dz = None
    if want_grad:
        dx, dy, dz = empty(B, n, like=Q), empty(B, m, like=Q), empty(B, m, like=Q)
    if split:
        ws = kkt_resgrad_ws(B, n, m, Q.device) if ws is None else ws
        _abi.call("iadmm_loss_grad_split", B, n, m, _p(Q), _p(p), _p(A0), _p(x), _p(y), _p(z), _p(cp), _p(cd),
                  _p(pr), _p(du), _p(dx), _p(dy), _p(dz), _p(ws), ws.numel() * 4, _stream())
    else:
        _abi.call("iadmm_loss_grad", B, n, m, _p(Q), _p(p), _p(A0), _p(x), _p(y), _p(z), _p(cp), _p(cd), _p(pr),
                  _p(du), _p(dx), _p(dy), _p(dz), _stream())
    return pr, du, dx, dy, dz
