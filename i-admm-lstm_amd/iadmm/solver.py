"""Fused test-mode solve loop (the hot path of main.py --test, main.py:818-1031).

One call = Ruiz scaling -> T Stage-I iterations -> final unscale -> final metrics, for one batch
of instances that is already resident in HBM.  Every step is a HIP kernel from libiadmm.so on
the current stream; no host synchronisation happens inside (metrics are kept on the device and
copied once at the end when ``history`` is requested).

Per iteration t (4 launches):
  iadmm_schedule      rho/alpha scalars of step t            models/lstm.py:60-63
  iadmm_kkt_resgrad   g = K^T (K xv - b~), implicit K        models/lstm.py:67-72
  iadmm_lstm_cell_fwd gates on fp32 MFMA + cell + projection models/lstm.py:74-80
  iadmm_admm_update   xv, x, z, y updates                    models/lstm.py:80-94
Buffers: x/y/z/xv and H ping-pong between two sets owned by the solver; C is updated in place.
"""
from __future__ import annotations

import torch

from . import ops

PARAM_NAMES = tuple(f"{a}_{g}" for g in "ifou" for a in ("W", "U", "b")) + ("W_h", "b_h", "rho", "alpha")


def param_dict(model_or_dict):
    if isinstance(model_or_dict, dict):
        return {k: model_or_dict[k] for k in PARAM_NAMES}
    return {k: getattr(model_or_dict, k) for k in PARAM_NAMES}


class PackedWeights:
    """Cell-kernel weight layout, re-packed only when a parameter changes (in-place updates bump
    ``_version``; replacing a tensor changes its data_ptr)."""

    def __init__(self):
        self._key = self._key16 = None
        self.Upk = self.Wx = self.Upk16 = self.wscale = None

    @staticmethod
    def _version_key(params, h):
        return tuple((params[k].data_ptr(), params[k]._version) for k in PARAM_NAMES[:13]) + (h,)

    def get(self, params, h):
        key = self._version_key(params, h)
        if key != self._key:
            with torch.no_grad():
                self.Upk, self.Wx = ops.lstm_pack(params, h)
            self._key = key
        return self.Upk, self.Wx

    def get_ucat_packed(self, params, h):
        """U_cat = [U_i U_f U_o U_u] ([h, 4h]) in gemm_nt_packed's tile layout: the A operand of
        the backward's dH = dP U_cat^T (re-packed when a parameter changes)."""
        key = self._version_key(params, h)
        if key != getattr(self, "_key_ucat", None):
            with torch.no_grad():
                ucat = torch.cat([params["U_" + k].detach() for k in "ifou"], dim=1).contiguous()
                self.Ucat_pk = ops.gemm_pack_a(ucat)
            self._key_ucat = key
        return self.Ucat_pk

    def get_f16x3(self, params, h):
        """Split weights of the optional f16x3 cell: (Upk16, wscale, Wx)."""
        _, Wx = self.get(params, h)
        key = self._version_key(params, h)
        if key != self._key16:
            with torch.no_grad():
                self.Upk16, self.wscale = ops.lstm_pack_f16x3(params, h)
            self._key16 = key
        return self.Upk16, self.wscale, Wx


class Timer:
    """hipEvent brackets on the current stream (named spans, summed).  Spans of one name may run
    on several streams at once (solve(lanes > 1)); :meth:`busy_ms` gives the time during which
    at least one of them was running."""

    def __init__(self, enabled):
        self.enabled = enabled
        self.spans = {}
        self.ref = None  # first event recorded: the time origin of busy_ms

    def start(self, name):
        if not self.enabled:
            return None
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        if self.ref is None:
            self.ref = ev
        return (name, ev)

    def stop(self, tok):
        if tok is None:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.spans.setdefault(tok[0], []).append((tok[1], ev))

    def totals_ms(self):
        torch.cuda.synchronize()
        return {k: sum(a.elapsed_time(b) for a, b in v) for k, v in self.spans.items()}

    def stats_ms(self, name):
        """(count, mean ms) of one span name."""
        torch.cuda.synchronize()
        v = self.spans.get(name, [])
        if not v:
            return 0, float("nan")
        return len(v), sum(a.elapsed_time(b) for a, b in v) / len(v)

    def busy_ms(self, name):
        """Length of the union of the intervals of span ``name`` (ms): equal to the summed
        durations when the spans never overlap (one stream)."""
        torch.cuda.synchronize()
        iv = sorted((self.ref.elapsed_time(a), self.ref.elapsed_time(b)) for a, b in self.spans.get(name, []))
        tot, end = 0.0, float("-inf")
        for a, b in iv:
            if a > end:
                tot += b - a
                end = b
            elif b > end:
                tot += b - end
                end = b
        return tot

    def reset(self):
        self.spans = {}
        self.ref = None


PRECISIONS = ("f32", "f16x3")


def lanes_for(B):
    """Default number of instance lanes of :func:`solve`: one.  Two staggered lanes measured +1.0 %
    at the bench shape (130.7 against 129.4 instances/s on one box): the residual-matvec
    workgroups (40 KiB of LDS) displace one of the cell kernel's two workgroups on a CU while they
    run, so only part of the matvec hides behind the other lane's cell kernel."""
    return 1


def solve(params, Q, p, A0, zl, zu, num_ineq, num_eq, T, sigma, scaling=True, scaling_iters=10,
          keep_unscaled=True, history=False, packed=None, timer=None, iter_hook=None, precision="f32",
          lanes=None):
    """Solve one batch; returns a dict with unscaled x/y/z, scaled state, final residuals.

    ``lanes``: the batch is cut into this many contiguous instance groups, each iterated on its own
    HIP stream (default :func:`lanes_for`; 1 with ``history``).  Instances are independent and
    every kernel is batch-invariant, so the result is bitwise the same for any lane count; the
    point is overlap: while one lane runs the MFMA-bound cell kernel, another's HBM-bound residual
    matvec and update kernels run beside it instead of in the cell kernels' gaps.

    Q[B,n,n], p[B,n,1], A0[B,m,n], zl/zu[B,m,1] fp32 device tensors (unscaled, Q already *2 as
    main.py:718 loads it).  ``keep_unscaled=False`` scales the data in place (saves 8 GB at the
    bench config) and reports residuals through the scaling identity instead of the originals.
    ``history=True`` records per-iteration obj / ls_res / primal / dual on the device and calls
    ``iter_hook(t, x, y, z)`` with the unscaled iterate ([B,n], [B,m], [B,m]) after each step.
    ``precision="f16x3"`` runs the gate GEMM on the fp16 matrix cores with the 3-term split of
    csrc/lstm_f16x3.hip (optional mode; the default "f32" is the fp32-MFMA path): H is carried as
    its two fp16 planes between iterations and the fp32 H is written on the last iteration.
    """
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {PRECISIONS}")
    f16 = precision == "f16x3"
    params = param_dict(params)
    B, n = Q.shape[0], Q.shape[1]
    m = A0.shape[1]
    if num_ineq + num_eq != m:
        raise ValueError(f"num_ineq + num_eq = {num_ineq + num_eq} but A0 has {m} rows")
    h = params["U_i"].shape[0]
    if T > params["rho"].shape[0]:
        raise ValueError(f"T={T} exceeds the model length {params['rho'].shape[0]} (models/lstm.py:60)")
    dev = Q.device
    N = n + m
    timer = timer or Timer(False)
    packed = packed or PackedWeights()
    if f16:
        Upk16, wscale, Wx = packed.get_f16x3(params, h)
    else:
        Upk, Wx = packed.get(params, h)
    rho_p, alpha_p, b_h = (params[k].detach().contiguous() for k in ("rho", "alpha", "b_h"))

    f32 = dict(dtype=torch.float32, device=dev)
    tok = timer.start("scaling")
    if scaling:
        dst = None if keep_unscaled else (Q, p, A0, zl, zu)
        Qs, ps, As, zls, zus, D, E, c = ops.ruiz_scale(Q, p, A0, zl, zu, scaling_iters, out=dst)
    else:
        Qs, ps, As, zls, zus = Q, p, A0, zl, zu
        D = E = c = None
    timer.stop(tok)

    # state (two sets) and work buffers
    tok = timer.start("untimed:setup")  # the reference allocates its zeros before start_time (main.py:836-841)
    xs = [torch.zeros(B, n, **f32), torch.empty(B, n, **f32)]
    ys = [torch.zeros(B, m, **f32), torch.empty(B, m, **f32)]
    zs = [torch.zeros(B, m, **f32), torch.empty(B, m, **f32)]
    xvs = [torch.zeros(B, N, **f32), torch.empty(B, N, **f32)]
    if f16:  # the fp32 H is written on the last iteration only (split planes per lane below)
        Hs = [torch.zeros(B, N, h, **f32)] * 2
    else:
        Hs = [torch.zeros(B, N, h, **f32), torch.empty(B, N, h, **f32)]
    C = torch.zeros(B, N, h, **f32)
    g = torch.empty(B, N, **f32)
    pv, zlv, zuv = ps.reshape(B, n), zls.reshape(B, m), zus.reshape(B, m)
    if history:
        hist = torch.zeros(4, T, B, **f32)  # obj, ls_res, primal, dual
        tmp = (torch.empty(B, n, **f32), torch.empty(B, m, **f32), torch.empty(B, m, **f32))
        lanes = 1
    timer.stop(tok)
    L = max(1, min(int(lanes if lanes is not None else lanes_for(B)), B))

    # lane streams and the KKT workspaces: the reference's model() would pay for its own work
    # buffers inside the timed call, so this stays in the timed scope
    tok = timer.start("setup")

    main = torch.cuda.current_stream(dev)
    lane = []  # per lane: instance slice, stream, its own scalars / projection partials / KKT workspace
    for i in range(L):
        b0 = (B * i) // L
        b1 = (B * (i + 1)) // L
        nb = b1 - b0
        strm = main if i == 0 else torch.cuda.Stream(device=dev)
        ln = dict(sl=slice(b0, b1), stream=strm,
                  scal=torch.empty(ops.NSCAL, **f32), part=torch.empty(ops.lstm_ntiles(h), nb * N, **f32),
                  kws=ops.kkt_resgrad_ws(nb, n, m, dev))
        if f16:  # split planes of H (ping-pong)
            f16t = dict(dtype=torch.float16, device=dev)
            ln["H16"] = [torch.zeros(2, nb, N, h, **f16t), torch.empty(2, nb, N, h, **f16t)]
        lane.append(ln)
    scal = lane[0]["scal"]
    timer.stop(tok)
    if L > 1:  # the lanes start after the scaling and the zero-fills on the main stream
        ready = main.record_event()
        for ln in lane:
            if ln["stream"] is not main:
                ln["stream"].wait_event(ready)
    # Lane i starts one residual-matvec later than lane i-1 (it waits for that lane's first KKT
    # launch).  Started together, the lanes run in lockstep (their cell kernels share the chip
    # evenly and end together, so their matvecs meet again); staggered, every lane's matvec and
    # update run while the other lanes' cell kernels run, and the offset persists.  (A high-priority
    # stream for lane 0 instead measured no better: profiles/r02_lanes.txt.)

    def iterate(ln, t, cur, nxt):
        sl, sc, part = ln["sl"], ln["scal"], ln["part"]
        ops.schedule(rho_p, alpha_p, t, out=sc)
        k = timer.start("k:kkt_resgrad")
        ops.kkt_resgrad(Qs[sl], As[sl], pv[sl], xs[cur][sl], ys[cur][sl], zs[cur][sl], xvs[cur][sl], sigma, sc,
                        num_ineq, g=g[sl], ws=ln["kws"])
        timer.stop(k)
        if t == 0 and L > 1:
            ln["kkt0"] = torch.cuda.current_stream(dev).record_event()
        k = timer.start("k:lstm_cell")
        if f16:
            H16 = ln["H16"]
            ops.lstm_cell_f16x3(H16[cur], C[sl], xvs[cur][sl], g[sl], Upk16, wscale, Wx, Hn16=H16[nxt], Cn=C[sl],
                                part=part, Hn=Hs[0][sl] if t == T - 1 else None)
        else:
            ops.lstm_cell(Hs[cur][sl], C[sl], xvs[cur][sl], g[sl], Upk, Wx, Hn=Hs[nxt][sl], Cn=C[sl], part=part)
        timer.stop(k)
        ops.admm_update(n, m, num_ineq, part, b_h, xvs[cur][sl], xs[cur][sl], ys[cur][sl], zs[cur][sl], zlv[sl],
                        zuv[sl], sc, out=(xvs[nxt][sl], xs[nxt][sl], ys[nxt][sl], zs[nxt][sl]))

    cur = 0
    # timed scope = the reference's model() calls (main.py:881-890): with history the per-iteration
    # metric work runs in "hist:" spans that the CLI's Parallel Time leaves out
    tok = timer.start("iterations") if not history else None
    for t in range(T):
        nxt = 1 - cur
        if history:
            tok = timer.start("iterations")
        if L == 1:
            iterate(lane[0], t, cur, nxt)
        else:
            for i, ln in enumerate(lane):  # enqueued round-robin; the lanes' streams run concurrently
                with torch.cuda.stream(ln["stream"]):
                    if t == 0 and i > 0:
                        ln["stream"].wait_event(lane[i - 1]["kkt0"])
                    iterate(ln, t, cur, nxt)
        if history:  # main.py:949-957 on unscaled data; kept on device
            timer.stop(tok)
            htok = timer.start("hist:metrics")
            ops.kkt_lsres(Qs, As, pv, xs[cur], ys[cur], zs[cur], xvs[nxt], sigma, scal, num_ineq,
                          out=hist[1, t])
            if scaling:
                ux, uy, uz = ops.unscale(D, E, c, xs[nxt], ys[nxt], zs[nxt], out=tmp)
            else:
                ux, uy, uz = xs[nxt], ys[nxt], zs[nxt]
            o, pr, du = _metrics(Q, p, A0, Qs, ps, As, D, E, c, ux, uy, uz, xs[nxt], ys[nxt], zs[nxt],
                                 keep_unscaled or not scaling)
            hist[0, t].copy_(o)
            hist[2, t].copy_(pr)
            hist[3, t].copy_(du)
            if iter_hook is not None:  # extra per-iteration device metrics (main.py:959-978)
                iter_hook(t, ux, uy, uz)
            timer.stop(htok)
        cur = nxt
    for ln in lane:  # join: everything after (and every buffer's release) orders after the lanes
        if ln["stream"] is not main:
            main.wait_stream(ln["stream"])
    if not history:
        timer.stop(tok)

    tok = timer.start("unscale")
    if scaling:
        x, y, z = ops.unscale(D, E, c, xs[cur], ys[cur], zs[cur])
    else:
        x, y, z = xs[cur], ys[cur], zs[cur]
    timer.stop(tok)

    tok = timer.start("untimed:metrics")  # the reference times no metric work (main.py:949-978)
    obj, pr, du = _metrics(Q, p, A0, Qs, ps, As, D, E, c, x, y, z, xs[cur], ys[cur], zs[cur],
                           keep_unscaled or not scaling)
    timer.stop(tok)
    out = dict(x=x.unsqueeze(-1), y=y.unsqueeze(-1), z=z.unsqueeze(-1), xv=xvs[cur].unsqueeze(-1),
               H=Hs[0] if f16 else Hs[cur], C=C, x_scaled=xs[cur].unsqueeze(-1), y_scaled=ys[cur].unsqueeze(-1),
               z_scaled=zs[cur].unsqueeze(-1), obj=obj, primal=pr, dual=du, scal=scal,
               scaled=(Qs, ps, As, zls, zus), D=D, E=E, c=c)
    if history:
        out.update(hist_obj=hist[0], hist_ls_res=hist[1], hist_primal=hist[2], hist_dual=hist[3])
    return out


def _metrics(Q, p, A0, Qs, ps, As, D, E, c, x, y, z, xh, yh, zh, have_unscaled):
    """Residuals on the unscaled problem (utils.py:53-54, 68-71).  Without the unscaled originals
    the scaled data give the same quantities through the scaling identities
      A0 x - z = E^-1 (Â x̂ - ẑ),  Qx + p + A0^T y = c^-1 D^-1 (Q̂ x̂ + p̂ + Â^T ŷ),  obj = c^-1 obĵ
    (equal in exact arithmetic; rounding differs)."""
    B, n = Qs.shape[0], Qs.shape[1]
    if have_unscaled:
        return ops.metrics(Q, p.reshape(B, n), A0, x, y, z)
    m = As.shape[1]
    obj_s, _, _ = ops.metrics(Qs, ps.reshape(B, n), As, xh, yh, zh)
    prim = (ops.bmv(As, xh) - zh) / E
    Aty = ops.kkt_matvec(Qs, As, torch.cat([torch.zeros_like(xh), yh], 1), 0.0, _unit_scal(Qs), m,
                         transpose=True)[:, :n]
    dual = ((ops.bmv(Qs, xh) + ps.reshape(B, n)) + Aty) / (c.reshape(B, 1) * D)
    return obj_s / c, prim.norm(dim=1), dual.norm(dim=1)


def _unit_scal(like):
    s = torch.ones(ops.NSCAL, dtype=torch.float32, device=like.device)
    return s


STAGE2_ALPHA = 1.6  # models/lu.py:24


def rho_rows_of(scal, B, m, num_ineq):
    """Per-row rho [B,m] of a two-class schedule (models/lstm.py:61-62)."""
    idx = torch.arange(m, device=scal.device)
    row = torch.where(idx < num_ineq, scal[ops.S_RHO_IN], scal[ops.S_RHO_EQ])
    return row.unsqueeze(0).expand(B, m).contiguous()


def fixed_alpha_scal(alpha, device):
    """Iteration scalars carrying only a fixed relaxation (Stage II): alpha, fl32(1 - alpha)."""
    a = torch.tensor(alpha, dtype=torch.float32)
    s = torch.zeros(ops.NSCAL, dtype=torch.float32)
    s[ops.S_ALPHA] = a
    s[ops.S_1MALPHA] = 1.0 - a
    return s.to(device)


def stage2_chunk(B, N, budget_bytes=None):
    """Instances per Stage-II factorisation chunk: the dense K is 4 N^2 bytes per instance
    (205 GB at config 4's N = 10000, B = 512), so the batch is factored in chunks that fit
    ``budget_bytes`` (default: 80 % of the device's free memory).  Instances are independent, so
    chunking changes nothing in the results."""
    if budget_bytes is None:  # free device memory + what torch's caching allocator holds unused
        free, _ = torch.cuda.mem_get_info()
        cached = torch.cuda.memory_reserved() - torch.cuda.memory_allocated()
        budget_bytes = int(0.8 * (free + cached))
    per = 4 * N * N + 64 * N  # K (factored in place) + pivots, rhs, solution, iterates
    cap = max(1, min(B, budget_bytes // per))
    # equal chunks, rounded up to whole multiples of the CU count when that adds no chunk: the
    # panel kernels run one workgroup per instance, so 512 instances as 410 + 102 take three
    # rounds of panels per column and as 256 + 256 two (the other kernels are throughput-bound)
    nch = -(-B // cap)
    step = -(-B // nch)
    cus = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count \
        if torch.cuda.is_available() else 0
    if cus and step > cus and -(-step // cus) * cus <= cap:
        step = -(-step // cus) * cus
    return step


def stage2(Q, p, A0, zl, zu, rho_rows, x, y, z, sigma, iters, alpha=STAGE2_ALPHA, timer=None, iter_hook=None,
           history=False, chunk=None):
    """Stage II feasibility restoration (models/lu.py:13-47, driver main.py:1035-1066):
    factor K once (rho of the last Stage-I iteration), then ``iters`` exact ADMM steps with
    alpha-relaxation on x and z.  Works on the unscaled data like the reference.
    Q[B,n,n], p[B,n], A0[B,m,n], zl/zu/rho_rows[B,m], x[B,n], y/z[B,m].  Returns the iterates and
    the factors (LU, piv) of the last chunk.  A singular K raises (like models/lu.py's torch.lu
    check).  The batch is processed in chunks of ``chunk`` instances (default
    :func:`stage2_chunk`: as many dense K as fit in memory).
    ``history=True`` records per-iteration obj / ls_res / primal / dual [4, iters, B] on the device
    (main.py:1068-1076: ls_res = ||K xv - b~|| with the solve's own K and b~) and
    ``iter_hook(t, x, y, z, sl)`` runs after every iteration on the instances ``sl`` of the batch;
    both in "hist:" timer spans."""
    timer = timer or Timer(False)
    B, n = x.shape
    m = y.shape[1]
    N = n + m
    scal = fixed_alpha_scal(alpha, x.device)
    hist = torch.zeros(4, iters, B, dtype=torch.float32, device=x.device) if history else None
    step = int(chunk) if chunk else stage2_chunk(B, N)
    xo, yo, zo = torch.empty_like(x), torch.empty_like(y), torch.empty_like(z)
    xvo = torch.empty(B, N, dtype=x.dtype, device=x.device)
    LU = piv = info = None
    for s0 in range(0, B, step):
        sl = slice(s0, min(B, s0 + step))
        Qc, pc, Ac, zlc, zuc, rc = (t[sl] for t in (Q, p, A0, zl, zu, rho_rows))
        xc, yc, zc = x[sl], y[sl], z[sl]
        LU = piv = None  # the previous chunk's factors are released before the next K is built
        tok = timer.start("stage2_assemble")
        K = ops.kkt_assemble(Qc, Ac, sigma, None, 0, rho_rows=rc)
        timer.stop(tok)
        tok = timer.start("stage2_factor")
        LU, piv, info = ops.lu_factor(K)
        timer.stop(tok)
        bad = int(info.max())  # one host read per factorisation
        if bad:
            raise RuntimeError(f"Stage II LU: U({bad},{bad}) is exactly zero (singular KKT matrix)")
        del K
        xv = None
        for t in range(iters):
            tok = timer.start("stage2_iterations")
            b = ops.kkt_rhs(pc, xc, yc, zc, sigma, rho_rows=rc)
            xs = ops.lu_solve(LU, piv, b)
            xv, xc, yc, zc = ops.admm_update(n, m, 0, None, None, xs, xc, yc, zc, zlc, zuc, scal, relax_z=True,
                                             rho_rows=rc)
            timer.stop(tok)
            if history or iter_hook is not None:
                htok = timer.start("hist:stage2")
                if history:
                    r = ops.kkt_matvec(Qc, Ac, xv, sigma, None, 0, rho_rows=rc) - b
                    hist[1, t, sl] = r.norm(dim=1)
                    o, pr, du = ops.metrics(Qc, pc, Ac, xc, yc, zc)
                    hist[0, t, sl] = o
                    hist[2, t, sl] = pr
                    hist[3, t, sl] = du
                if iter_hook is not None:
                    iter_hook(t, xc, yc, zc, sl)
                timer.stop(htok)
        xo[sl], yo[sl], zo[sl] = xc, yc, zc
        if xv is not None:
            xvo[sl] = xv
    out = dict(x=xo, y=yo, z=zo, xv=xvo if iters > 0 else None, LU=LU, piv=piv, info=info, chunk=step)
    if history:
        out.update(hist_obj=hist[0], hist_ls_res=hist[1], hist_primal=hist[2], hist_dual=hist[3])
    return out
