"""Benchmark: QP instances/s of the I-ADMM-LSTM test-mode solve at BASELINE config 2.

A "step" = one full test-mode solve of the per-GPU batch, already resident in HBM (the timed
scope of main.py:825-834,881-890,1024-1031): Ruiz scaling (10 rounds) -> K=100 Stage-I
iterations -> final unscale.  Instances: n=1000, 500 inequality + 500 equality rows, hidden 800,
B=1024 per GPU (synthetic, restating generate_data.py:67-76).  Weights: the checkpoint
``checkpoints/QP_{n}_{eq}_{ineq}_{T}_{h}.pth`` (main.py's naming; the reference's own training recipe,
scripts/Synthetic.sh:3, run through this repo's main.py train mode -- the epoch-61 save, adopted in
r05 after passing the K = 100 fp64 envelope, checkpoints/README.md) when it exists, else random init
with the reference's initialisation.  Throughput does not depend on weight values; the final residual does (the
random-init solve diverges at this shape), so both are reported when a checkpoint is used.

Multi-GPU: one process per GPU (torch.distributed.run); the instance batch is sharded (rank r
solves instances [r*B, (r+1)*B)) with no data-path collective; a barrier brackets the timed
region and the max time over ranks is reported ("scaling": "weak").

Prints ONE JSON line on rank 0, including
  roofline      the dominant kernel (iadmm_lstm_cell_fwd, fp32 MFMA) from hipEvent timing of
                every launch inside the timed region, plus the same for the HBM-bound residual
                matvec (iadmm_kkt_resgrad) under "roofline_matvec";
  cpu_baseline  the CPU oracle (oracle/iadmm_oracle.py: the reference's op structure in
                PyTorch-CPU fp32) on a bounded sample of the same workload, rank 0 only, with
                a parity block: the GPU's result on the SAME instances against the oracle's
                (x, y, z rel-L2, primal/dual relative error, K = outer_T iterations).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "i-admm-lstm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md, Peak FP32 (matrix), spec
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md, HBM3E peak BW, spec
KKT_KERNELS = ("kkt_split_p1", "kkt_split_c1", "kkt_split_p2", "kkt_split_c2")  # iadmm_kkt_resgrad


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=1024, help="instances per GPU")
    ap.add_argument("--num_var", type=int, default=1000)
    ap.add_argument("--num_ineq", type=int, default=500)
    ap.add_argument("--num_eq", type=int, default=500)
    ap.add_argument("--hidden_dim", type=int, default=800)
    ap.add_argument("--outer_T", type=int, default=100)
    ap.add_argument("--sigma", type=float, default=6e-6)
    ap.add_argument("--cpu-sample", type=int, default=8,
                    help="instances in the CPU baseline (0: skip).  8 of config 1's 64: the CPU cost is "
                         "linear in the batch (batched ops, no cross-instance work), and 64 would take "
                         "~4 min of CPU time, beyond the bench's bounded-sample budget")
    ap.add_argument("--weights", type=str, default="auto",
                    help="'auto' (the checkpoint under checkpoints/ when present, else random init), "
                         "'random', or a .pth path")
    ap.add_argument("--alt-f16x3", type=int, default=1,
                    help="also time one step of the optional split-precision cell (reported under "
                         "'alt_precision', never as the headline value)")
    ap.add_argument("--lanes", type=int, default=0,
                    help="instance lanes (HIP streams) of the solve; 0: solver.lanes_for(batch)")
    ap.add_argument("--stage2-iters", type=int, default=20,
                    help="feas_rest_num of a Stage II run (models/lu.py via main.py:1035-1066) on the solved "
                         "batch, timed and reported under 'stage2' (0: skip)")
    ap.add_argument("--train-batch", type=int, default=512,
                    help="instances per GPU of the training record (BASELINE config 5: 4096 over 8 GPUs; "
                         "one warm-up + one timed TBPTT window of outer_T iterations; 0: skip)")
    ap.add_argument("--train-micro-batch", type=int, default=128)
    ap.add_argument("--in-place-scaling", action="store_true",
                    help="scale Q/A0 in place (no unscaled copy; residuals via the scaling identity)")
    a = ap.parse_args()
    if a.in_place_scaling and a.warmup + a.steps == 1 and a.cpu_sample > 0:
        ap.error("a single in-place step keeps no unscaled copy for the CPU baseline: add --cpu-sample 0")
    return a


def pmc_traffic(kernel_prefix, n, m, h, B, lanes=1):
    """HBM-side bytes of one operation per iteration of the whole batch (the sum over the kernels
    whose names contain one of ``kernel_prefix``, times the lanes: one dispatch per lane) from the
    committed rocprofv3 --pmc summaries of this exact workload (tools/pmc_summary.py output, one
    FETCH_SIZE and one WRITE_SIZE pass; file suffix ``_L{lanes}`` when lanes > 1).
    gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts 128-B requests at 64 B, so
    it is doubled; WRITE_SIZE is taken as is.  Returns (bytes, [the profile files used]), or
    (None, None) when no matching profile exists."""
    import csv
    import glob
    tot, used = 0.0, []
    for ctr, mult in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        sfx = f"_L{lanes}" if lanes > 1 else ""
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{ctr}_n{n}_m{m}_h{h}_B{B}{sfx}.csv")))
        if not files:
            return None, None
        names = (kernel_prefix,) if isinstance(kernel_prefix, str) else kernel_prefix
        rows = [r for r in csv.DictReader(open(files[-1]))
                if any(k in r["kernel"] for k in names) and r["counter"] == ctr]
        if not rows:
            return None, None
        # one launch of the operation = one dispatch of every kernel it consists of
        tot += mult * sum(float(r["mean"]) for r in rows) * 1024.0 * lanes
        used.append(os.path.relpath(files[-1], ROOT))
    return tot, used


def rocprof_avg_ms(kernels, tag_glob="r*_bench_kernel_stats.csv"):
    """Sum of the rocprofv3 --stats average durations (ms) of ``kernels`` (name substrings) in the
    newest committed bench kernel-stats profile, with the file name; (None, None) without one."""
    import csv
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", tag_glob)))  # r01 < r02 < r02final < r03
    for f in reversed(files):
        rows = list(csv.DictReader(open(f)))
        got = {}
        for k in kernels:
            hit = [r for r in rows if k in r["Name"]]
            if hit:
                got[k] = float(hit[0]["AverageNs"]) / 1e6
        if len(got) == len(kernels):
            return sum(got.values()), os.path.relpath(f, ROOT)
    return None, None


def pmc_traffic_stage2(n, m, B):
    """HBM bytes of one factorization (every lu_* kernel but the solve) from the committed Stage-II
    PMC summaries of tools/profile_lu.py (one factorization; tools/pmc_summary.py: per-kernel mean
    per dispatch x dispatches), FETCH_SIZE x 2
    (gfx950 correction) + WRITE_SIZE; (bytes, [files used]) or (None, None) without a matching
    profile."""
    import csv
    import glob
    tot, used = 0.0, []
    for ctr, mult in (("FETCH_SIZE", 2.0), ("WRITE_SIZE", 1.0)):
        files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_stage2_pmc_{ctr}_N{n + m}_B{B}.csv")))
        if not files:
            return None, None
        rows = [r for r in csv.DictReader(open(files[-1]))
                if "iadmm::lu_" in r["kernel"] and "solve" not in r["kernel"] and r["counter"] == ctr]
        if not rows:
            return None, None
        # the profile run factors once (tools/profile_lu.py): every dispatch belongs to it
        tot += mult * sum(float(r["mean"]) * float(r["dispatches"]) for r in rows) * 1024.0
        used.append(os.path.relpath(files[-1], ROOT))
    return tot, used


def box_ceiling(local):
    """What THIS box delivers: the fp32 MFMA rate of a register-only
    v_mfma_f32_32x32x2_f32 stream on every SIMD (csrc/probe.hip, 2 workgroups of 4 waves per CU,
    ~40 ms per run, best of 3) and the HBM rate of a 1-GiB float4 copy (2 x bytes per launch,
    best of 10), both timed with hipEvents on the launch stream before the timed steps.  The
    rooflines report their fraction of these beside the fraction of the spec peaks."""
    from iadmm import _abi, ops
    cus = torch.cuda.get_device_properties(local).multi_processor_count
    blocks = 2 * cus
    out = torch.empty(blocks * 256, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        e1.synchronize()
        return e0.elapsed_time(e1)

    def mfma(iters):
        return timed(lambda: _abi.call("iadmm_probe_mfma", blocks, iters, out.data_ptr(), ops._stream()))

    mfma(1000)
    it = 20000
    it = max(1000, int(it * 40.0 / max(mfma(it), 1e-3)))
    flop = float(_abi.lib().iadmm_probe_mfma_flop(blocks, it))
    tflops = max(flop / (mfma(it) * 1e-3) / 1e12 for _ in range(3))
    nbytes = 1 << 30
    src = torch.ones(nbytes // 4, dtype=torch.float32, device="cuda")
    dst = torch.empty_like(src)

    def copy():
        return timed(lambda: _abi.call("iadmm_probe_copy", nbytes, src.data_ptr(), dst.data_ptr(), ops._stream()))

    copy()
    gbs = max(2.0 * nbytes / (copy() * 1e-3) / 1e9 for _ in range(10))
    ok = bool(torch.equal(dst[:1024], src[:1024]))
    del dst
    # r05: a read-only sweep too (the residual matvec is ~all reads; the copy alone measured below the
    # matvec's own read rate, so it was no ceiling for it): best over workgroups per CU and loads in
    # flight, 4 GiB (past the 256 MiB Infinity Cache many times over)
    rbytes = 4 << 30
    big = torch.ones(rbytes // 4, dtype=torch.float32, device="cuda")
    rout = torch.empty(32 * cus * 256, dtype=torch.float32, device="cuda")
    read = {}
    for wg in (2, 4, 8, 16):
        for un in (8, 16):
            fn = lambda: _abi.call("iadmm_probe_read", rbytes, big.data_ptr(), rout.data_ptr(), wg, un,  # noqa: E731
                                   ops._stream())
            timed(fn)
            read[f"{wg}x{un}"] = max(rbytes / (timed(fn) * 1e-3) / 1e9 for _ in range(3))
    best_read = max(read, key=read.get)
    del src, big, rout, out
    torch.cuda.empty_cache()
    hbm = max(gbs, read[best_read])
    return {"mfma_f32_tflops": tflops, "mfma_frac_of_spec": tflops / FP32_MFMA_PEAK_TFLOPS,
            "hbm_copy_gbs": gbs, "hbm_read_gbs": read[best_read], "hbm_read_shape": best_read,
            "hbm_gbs": hbm, "hbm_frac_of_spec": hbm / HBM_PEAK_GBS, "copy_checked": ok,
            "method": f"csrc/probe.hip: {blocks} x 256-thread workgroups x {it} x 8 register MFMAs "
                      f"(v_mfma_f32_32x32x2_f32), best of 3; float4 copy of 1 GiB, best of 10; float4 "
                      f"read sweep of 4 GiB, best of 3 at each of (workgroups per CU) x (loads in flight) "
                      f"{sorted(read)}; hbm_gbs = the larger of copy and read; hipEvents"}


def baseline_config(args, world):
    shape = (args.num_var, args.num_ineq, args.num_eq, args.hidden_dim, args.outer_T, args.batch)
    if shape == (1000, 500, 500, 800, 100, 1024):
        return "BASELINE config 2" if world == 1 else "BASELINE config 3"
    if shape == (5000, 2500, 2500, 2048, 200, 512):
        return "BASELINE config 4"
    return "custom shape"


def cpu_model():
    """Host CPU model name (/proc/cpuinfo), for the cpu_baseline record."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


PARITY_TOL = {"x": 1e-4, "z": 1e-4, "y": 5e-3, "primal": 1e-4, "dual": 1e-4}
"""Stated fp32 tolerance of the GPU-vs-oracle comparison (SURVEY.md §8(c) contract: rel-L2(x^K)
and primal/dual relative error <= 1e-4; y <= 5e-3 because the equality-row update
y = rho_eq (z~ - b) with rho_eq ~ 500 cancels ~3 digits, DESIGN.md §4).  Divergent dynamics
(random-init weights at this shape) amplify rounding differences, so that regime is reported
but not held to the tolerance."""


def parity(gpu, ref, Bc):
    """GPU result of instances [0, Bc) against the oracle's on the same instances."""
    res = {}
    for k in ("x", "y", "z"):
        a = gpu[k][:Bc].reshape(Bc, -1).double().cpu()
        b = ref[k].reshape(Bc, -1).double()
        res[k + "_rel_l2"] = float(((a - b).norm(dim=1) / b.norm(dim=1).clamp_min(1e-30)).max())
    for k in ("primal", "dual"):
        a = gpu[k][:Bc].reshape(-1).double().cpu()
        b = ref[k].reshape(-1).double()
        res[k + "_max_rel"] = float(((a - b).abs() / b.abs().clamp_min(1e-30)).max())
        res[k + "_mean_gpu"] = float(a.mean())
        res[k + "_mean_cpu"] = float(b.mean())
    res["tol"] = PARITY_TOL
    res["within_tol"] = all(res[k + ("_rel_l2" if k in "xyz" else "_max_rel")] <= v for k, v in PARITY_TOL.items())
    return res


def run_oracle(args, cpu, params):
    from oracle import iadmm_oracle as orc
    pc = {k: v.detach().cpu() for k, v in params.items()}
    t0 = time.perf_counter()
    with torch.no_grad():
        out = orc.solve(pc, cpu["Q"], cpu["p"], cpu["A0"], cpu["zl"], cpu["zu"], args.num_ineq, args.num_eq,
                        args.outer_T, args.sigma, args.hidden_dim)
    return out, time.perf_counter() - t0


def cpu_baseline(args, d, params, gpu_out, weights_tag, extra=()):
    """Oracle (reference op structure, torch-CPU fp32) on the first ``cpu_sample`` instances, timed
    (the baseline) and compared with the GPU's result on the same instances (parity).  ``extra``:
    further (tag, params, gpu_out) sets checked for parity only (untimed)."""
    Bc = args.cpu_sample
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    cpu = {k: d[k][:Bc].cpu() for k in ("Q", "p", "A0", "zl", "zu")}
    out, dt = run_oracle(args, cpu, params)
    rec = dict(value=Bc / dt, unit="QP instances/s", cores=threads, kind="port", cpu_model=cpu_model(),
               cores_note=f"torch.set_num_threads({threads}) from OMP_NUM_THREADS: the GPU box sets it to the CPU "
                          f"share of one GPU's lease (16); os.cpu_count() = {os.cpu_count()} counts the whole host",
               sample=f"{Bc} instances x full solve (Ruiz + K={args.outer_T} + unscale), the same synthetic "
                      f"instances 0..{Bc - 1} and weights ({weights_tag}) as the GPU run, {dt:.1f} s; "
                      + (f"{Bc} of config 1's 64 instances (CPU cost is linear in the batch; all 64 timed once: "
                         "profiles/r05_cpu_leg_64.json)" if Bc < 64 else "all 64 of config 1's instances"),
               final_primal=float(out["primal"].mean()), final_dual=float(out["dual"].mean()),
               parity={weights_tag: parity(gpu_out, out, Bc)})
    for tag, prm, gout in extra:
        o, _ = run_oracle(args, cpu, prm)
        rec["parity"][tag] = parity(gout, o, Bc)
    return rec


def stage2_record(args, d, out, n, mi, me, B):
    """Time Stage II (solver.stage2: dense K, batched blocked LU, feas_rest_num solves) on the
    solved batch; per-phase hipEvent times and instances/s."""
    from iadmm import solver
    m = mi + me
    rho_rows = solver.rho_rows_of(out["scal"], B, m, mi)
    x, y, z = (out[k].reshape(B, -1) for k in ("x", "y", "z"))
    st_args = (d["Q"], d["p"].reshape(B, n), d["A0"], d["zl"].reshape(B, m), d["zu"].reshape(B, m), rho_rows,
               x, y, z, args.sigma, args.stage2_iters)
    r = solver.stage2(*st_args)
    del r
    tm = solver.Timer(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = solver.stage2(*st_args, timer=tm)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    spans = tm.totals_ms()
    from iadmm import ops
    pr = ops.metrics(d["Q"], d["p"].reshape(B, n), d["A0"], r["x"], r["y"], r["z"])
    N = n + mi + me
    fac_ms = spans.get("stage2_factor")
    fac_flop = B * 2.0 / 3.0 * N ** 3
    fac_tf = fac_flop / (fac_ms * 1e-3) / 1e12
    st2_traffic, st2_src = pmc_traffic_stage2(n, mi + me, B)
    rec = {"value": B / el, "unit": "QP instances/s", "feas_rest_num": args.stage2_iters, "ms": 1e3 * el,
           "assemble_ms": spans.get("stage2_assemble"), "factor_ms": fac_ms,
           "solve_iter_ms": spans.get("stage2_iterations", 0.0) / args.stage2_iters,
           "roofline": {"kernel": "iadmm_lu_factor", "bound": "mfma", "achieved": fac_tf,
                        "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": fac_tf / FP32_MFMA_PEAK_TFLOPS,
                        "algorithmic_per_launch": fac_flop, "algorithmic": "2/3 N^3 per instance (getrf)",
                        "traffic": st2_traffic, "traffic_source": st2_src,
                        "traffic_note": "all LU kernels of one factorization (FETCH_SIZE x 2 + WRITE_SIZE, "
                                        "separate --pmc passes of tools/profile_lu.py)"},
           "chunk": r["chunk"], "final_primal_mean": float(pr[1].mean()), "final_dual_mean": float(pr[2].mean()),
           "note": "Stage II (--feas_rest) on the solved batch: K assembled from the last Stage-I rho on the "
                   "unscaled data, batched blocked LU (csrc/lu.hip) once, feas_rest_num solves + alpha=1.6 "
                   "updates; outside the headline's timed scope"}
    del r
    return rec


def train_record(args, d, mi, me, dist, world):
    """BASELINE config 5 per GPU: one TBPTT window (main.py:336-358: outer_T forward iterations +
    the residual loss + backward through all of them + gradient all-reduce + Adam step) on the
    first ``train_batch`` instances (Ruiz-scaled copy), micro-batched; one untimed warm-up window,
    one timed.  Per-kernel hipEvent spans of the training kernels (iadmm/autograd.TIMER) give the
    cell backward's MFMA roofline (its recompute GEMM = the forward's 8 N h^2 flop per
    instance-iteration, rocprof: profiles/*train*kernel_stats.csv)."""
    from iadmm import autograd, ops, solver, train
    from models.lstm import LSTM
    n = args.num_var
    N, h, T = n + mi + me, args.hidden_dim, args.outer_T
    Bt, mb = min(args.train_batch, d["Q"].shape[0]), args.train_micro_batch
    sc = ops.ruiz_scale(*(d[k][:Bt] for k in ("Q", "p", "A0", "zl", "zu")), 10)
    ds = dict(zip(("Q", "p", "A0", "zl", "zu"), sc[:5]))
    del sc
    torch.manual_seed(17)
    model = LSTM(mi + me, 2, h, T, "cuda")
    opt = torch.optim.Adam(model.parameters(), lr=5e-5)  # scripts/Synthetic.sh:3

    def window():
        return train.tbptt_batch(model, ds, mi, me, T, T, args.sigma, opt, micro_batch=mb, global_batch=world * Bt,
                                 dist=dist)

    window()
    torch.cuda.synchronize()
    tm = solver.Timer(True)
    autograd.TIMER = tm
    calls0 = train.ALLREDUCE_CALLS
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = window()
    torch.cuda.synchronize()
    el = parallel_max(time.perf_counter() - t0, dist)
    autograd.TIMER = None
    nb, ms_bwd = tm.stats_ms("k:cell_bwd")
    spans = {k[2:]: v for k, v in tm.totals_ms().items()}
    mrows = min(mb, Bt) * N                       # rows of one micro-batch launch
    flop = 8.0 * mrows * h * h                    # recompute GEMM of one cell-backward launch
    tf = flop / (ms_bwd * 1e-3) / 1e12
    del ds, model, opt
    return {"value": world * Bt / el, "unit": "training instances/s", "per_gpu": Bt / el,
            "batch_per_gpu": Bt, "micro_batch": mb, "outer_T": T, "truncated_length": T, "ms": 1e3 * el,
            "loss": loss, "allreduce_calls": train.ALLREDUCE_CALLS - calls0,
            "kernel_ms_per_window": spans,
            "roofline": {"kernel": "iadmm_lstm_cell_bwd", "bound": "mfma", "achieved": tf,
                         "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP32_MFMA_PEAK_TFLOPS,
                         "avg_launch_ms": ms_bwd, "launches": nb, "algorithmic_per_launch": flop,
                         "algorithmic": "8 N h^2 per instance-iteration (gate pre-activation recompute on MFMA); "
                                        "the epilogue's elementwise backward is not counted"},
            "note": "BASELINE config 5 per GPU (4096 instances over 8 GPUs = 512 each): one TBPTT window of "
                    "main.py:336-358 (forward + loss + backward + RCCL gradient all-reduce when N > 1 + Adam), "
                    "lr 5e-5 (scripts/Synthetic.sh:3), random init; outside the headline's timed scope"}


def parallel_max(v, dist):
    from iadmm import parallel
    return parallel.max_over_ranks(v, dist, device="cuda")


def load_weights(args, h, T):
    """(params dict on cuda, tag): the checkpoint named like main.py's (QP_{n}_{eq}_{ineq}_{T}_{h})
    under checkpoints/ for --weights auto, a given .pth, or random init."""
    from iadmm import data
    from iadmm.solver import PARAM_NAMES
    path = None
    if args.weights == "auto":
        cand = os.path.join(ROOT, "checkpoints", f"QP_{args.num_var}_{args.num_eq}_{args.num_ineq}_{T}_{h}.pth")
        path = cand if os.path.exists(cand) else None
    elif args.weights != "random":
        path = args.weights
    if path is None:
        return data.init_lstm_params(h, T, device="cuda"), "random-init"
    sd = torch.load(path, map_location="cuda", weights_only=True)
    params = {k: sd[k].float().contiguous() for k in PARAM_NAMES}
    if params["U_i"].shape[0] != h or params["rho"].shape[0] < T:
        raise SystemExit(f"{path}: hidden {params['U_i'].shape[0]} / length {params['rho'].shape[0]} "
                         f"do not fit hidden_dim={h}, outer_T={T}")
    return params, "trained:" + os.path.relpath(path, ROOT)


def launch_ranks(args):
    """``python bench.py --gpus N`` with no launcher around it and N > 1: run N ranks under
    torch.distributed.run as a child process and exit with its status (iadmm/launch.py; nothing
    here has touched the GPU yet).  Under a launcher, WORLD_SIZE must equal --gpus."""
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "iadmm_launch", os.path.join(ROOT, "i-admm-lstm_amd", "iadmm", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.relaunch(os.path.abspath(sys.argv[0]), sys.argv[1:], args.gpus)


def master_dev(d, master):
    """Unscaled instances on the device for the training record when the solve scaled in place."""
    if master is None:
        return d
    return {k: v.to("cuda") if v.device.type == "cpu" else v for k, v in master.items()}


def heartbeat(period_s=60.0):
    """Print a progress line to stderr every ``period_s`` while a long step runs (config 4 takes
    minutes per step; a silent process looks hung to a supervisor)."""
    import threading
    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(period_s)
            print(f"[bench] running, {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def main():
    args = parse()
    launch_ranks(args)
    heartbeat()
    from iadmm import data, parallel, solver
    world, rank, local = parallel.env()
    local, backend = parallel.device_and_backend(local)
    torch.cuda.set_device(local)
    dist = parallel.init(backend, local) if parallel.want_dist(world) else None
    box = box_ceiling(local)  # before any data is allocated (the copy takes 2 GiB)

    n, mi, me, h, T, B = args.num_var, args.num_ineq, args.num_eq, args.hidden_dim, args.outer_T, args.batch
    N = n + mi + me
    first, count = parallel.shard(world * B, world, rank)  # weak scaling: B instances per GPU
    d = data.make_qp_batch(n, mi, me, count, first_index=first, device="cuda")
    params, weights_tag = load_weights(args, h, T)
    packed = solver.PackedWeights()
    keep = not args.in_place_scaling
    if not keep and args.warmup + args.steps > 1:
        # restored before every step (untimed); on the host when a device copy would not fit
        # (config 4: Q and A0 are 102 GB per GPU)
        big = sum(v.numel() * 4 for v in d.values()) > 0.2 * torch.cuda.get_device_properties(local).total_memory
        master = {k: v.to("cpu" if big else v.device, copy=True) for k, v in d.items()}
    elif not keep:
        master = None

    lanes = args.lanes or solver.lanes_for(count)

    def step(timer, precision="f32", prm=None):
        if not keep and master is not None:
            for k in d:
                d[k].copy_(master[k])
            torch.cuda.synchronize()
        with torch.no_grad():
            return solver.solve(prm or params, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], mi, me, T, args.sigma,
                                keep_unscaled=keep, packed=None if prm else packed, timer=timer, precision=precision,
                                lanes=lanes)

    for _ in range(args.warmup):
        step(None)
    torch.cuda.synchronize()
    print(f"[bench] rank {rank} data + warmup ready", file=sys.stderr, flush=True)

    timer = solver.Timer(True)
    elapsed = 0.0
    step_times = []
    out = None
    for _ in range(args.steps):
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        out = None  # the previous step's state (H, C: 13 GB) is released before the next one allocates
        t0 = time.perf_counter()
        out = step(timer)
        torch.cuda.synchronize()
        step_times.append(time.perf_counter() - t0)
        elapsed += step_times[-1]
        print(f"[bench] rank {rank} step done, {step_times[-1]:.2f} s", file=sys.stderr, flush=True)
    elapsed_own = elapsed
    elapsed = parallel.max_over_ranks(elapsed, dist, device="cuda")
    primal, dual = float(out["primal"].mean()), float(out["dual"].mean())

    # dominant kernel and residual matvec, from the per-launch hipEvents of the timed steps.  With
    # several lanes the launches of one kernel overlap (each covers B / lanes instances), so the
    # achieved rate is the kernel's total algorithmic work over its busy time (the union of its
    # launch intervals); with one lane that is work per launch / mean launch time.
    n_cell, ms_cell = timer.stats_ms("k:lstm_cell")
    n_kkt, ms_kkt = timer.stats_ms("k:kkt_resgrad")
    busy_cell, busy_kkt = timer.busy_ms("k:lstm_cell"), timer.busy_ms("k:kkt_resgrad")
    spans = timer.totals_ms()
    cell_flop = B * (8.0 * N * h * h + 18.0 * N * h)            # per instance-batch iteration
    kkt_bytes = B * (2.0 * (n * n + (mi + me) * n) * 4 + 10.0 * N * 4)
    iters = args.steps * T
    cell_tf = cell_flop * iters / (busy_cell * 1e-3) / 1e12
    kkt_gbs = kkt_bytes * iters / (busy_kkt * 1e-3) / 1e9

    # Stage II (--feas_rest) on the solved batch, like main.py:1035-1066: K from the last Stage-I
    # rho on the unscaled data, factored once, then feas_rest_num exact iterations (one warm-up run,
    # one timed run; not part of the headline value, whose timed scope is the README test command)
    st2 = None
    if args.stage2_iters > 0 and keep:
        st2 = stage2_record(args, d, out, n, mi, me, B)

    # optional split-precision mode: one step after the headline steps, reported beside it
    alt = None
    if args.alt_f16x3 and h % 8 == 0 and (keep or master is not None):
        x32 = out["x"].clone()
        for k in ("H", "C"):
            out.pop(k, None)
        timer16 = solver.Timer(True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out16 = step(timer16, "f16x3")
        torch.cuda.synchronize()
        el16 = parallel.max_over_ranks(time.perf_counter() - t0, dist, device="cuda")
        n16, ms16 = timer16.stats_ms("k:lstm_cell")
        busy16 = timer16.busy_ms("k:lstm_cell")
        alt = {"mode": "f16x3",
               "note": "optional split-precision gate GEMM (3-term fp16 split, fp32 accumulation, "
                       "csrc/lstm_f16x3.hip); not the headline value",
               "value": world * B / el16, "unit": "QP instances/s", "ms_per_step": 1e3 * el16,
               "cell_avg_launch_ms": ms16, "cell_tflops_f32_equiv": cell_flop * T / (busy16 * 1e-3) / 1e12,
               "final_residual": {"primal_mean": float(out16["primal"].mean()),
                                  "dual_mean": float(out16["dual"].mean())},
               "x_rel_l2_vs_f32_run": float((out16["x"] - x32).norm() / x32.norm().clamp_min(1e-30))}
        del out16

    # the random-init weights' residual beside the trained one (untimed: same work, other values)
    rand = None
    if weights_tag != "random-init" and (keep or master is not None):
        prm_r = data.init_lstm_params(h, T, device="cuda")
        out_r = step(None, prm=prm_r)
        rand = (prm_r, {k: out_r[k] for k in ("x", "y", "z", "primal", "dual")})
        del out_r

    # BASELINE config 5 per GPU: one timed TBPTT training window (after the inference work; the
    # solve's state is released first: the window saves ~1.6 GB of activations per iteration at
    # micro-batch 128)
    trn = None
    mb_t = min(args.train_micro_batch, args.train_batch, count)
    act_bytes = 2.0 * 4 * mb_t * N * h * T  # saved H and C of every iteration of one micro-batch
    train_fits = act_bytes < 0.7 * torch.cuda.get_device_properties(local).total_memory
    if args.train_batch > 0 and train_fits:
        out_keep = {k: out[k] for k in ("x", "y", "z", "primal", "dual")}
        out = None
        torch.cuda.empty_cache()
        trn = train_record(args, d if keep else master_dev(d, master), mi, me, dist, world)
        out = out_keep
        torch.cuda.empty_cache()

    # the same roofline from the committed rocprof profile of this workload (another run: rocprof
    # serialises and times each of the four kernels; the hipEvent span above brackets them back to back)
    kkt_rocprof = None
    if (n, mi, me, h, B) == (1000, 500, 500, 800, 1024):
        ms_rp, src = rocprof_avg_ms(KKT_KERNELS)
        if ms_rp:
            gbs = kkt_bytes / (ms_rp * 1e-3) / 1e9
            kkt_rocprof = {"avg_launch_ms": ms_rp, "achieved": gbs, "frac": gbs / HBM_PEAK_GBS, "source": src}

    cell_traffic = pmc_traffic(("cell_fwd_dma_kernel",), n, mi + me, h, B, lanes)
    kkt_traffic = pmc_traffic(KKT_KERNELS, n, mi + me, h, B, lanes)
    # per-rank record (which GPU, which instances, how long): gathered to rank 0 (measurement only)
    ranks = parallel.gather_records(dict(rank=rank, first=first, count=count, elapsed_s=elapsed_own,
                                         step_s=step_times, box_mfma_tflops=box["mfma_f32_tflops"],
                                         box_hbm_gbs=box["hbm_gbs"], **parallel.device_record(local)), dist)

    res = None
    if rank == 0:
        total = world * B * args.steps
        res = {
            "metric": "QP instances/sec at n=1000 m=1000 K=100; final primal+dual residual",
            "value": total / elapsed,
            "unit": "QP instances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dist_backend": dist.get_backend() if dist else None,
            "dtype": "f32",
            "data": f"synthetic (generate_data.py:67-76 distribution, per-instance seeds); weights {weights_tag}",
            "config": {"workload": f"QP n={n} ineq={mi} eq={me} K={T} hidden={h} --test --scaling, "
                                   f"batch={B}/GPU ({baseline_config(args, world)}), {lanes} lane(s)",
                       "global_batch": world * B, "num_var": n, "num_ineq": mi, "num_eq": me,
                       "outer_T": T, "hidden_dim": h, "parallelism": f"instance-shard x{world}", "lanes": lanes,
                       "in_place_scaling": not keep},
            "final_residual": {"primal_mean": primal, "dual_mean": dual, "sum": primal + dual,
                               "weights": weights_tag},
            "roofline": {"kernel": "iadmm_lstm_cell_fwd", "bound": "mfma", "achieved": cell_tf,
                         "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": cell_tf / FP32_MFMA_PEAK_TFLOPS,
                         "traffic": cell_traffic[0], "traffic_source": cell_traffic[1],
                         "avg_launch_ms": ms_cell, "launches": n_cell, "busy_ms_per_iteration": busy_cell / iters,
                         "algorithmic_per_iteration": cell_flop,
                         "algorithmic_per_launch": cell_flop / lanes},
            "roofline_matvec": {"kernel": "iadmm_kkt_resgrad", "bound": "hbm", "achieved": kkt_gbs,
                                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": kkt_gbs / HBM_PEAK_GBS,
                                "traffic": kkt_traffic[0], "traffic_source": kkt_traffic[1],
                                "kernels": "kkt_split_p1 + c1 + p2 + c2 (row-block split, csrc/kkt.hip)",
                                "timing": "hipEvents around the four launches of each call, this run",
                                "rocprof": kkt_rocprof,
                                "avg_launch_ms": ms_kkt, "launches": n_kkt, "busy_ms_per_iteration": busy_kkt / iters,
                                "algorithmic_per_iteration": kkt_bytes,
                                "algorithmic_per_launch": kkt_bytes / lanes},
            "phase_ms_per_step": {k: v / args.steps for k, v in spans.items() if not k.startswith("k:")},
        }
        # the same fractions against what this box measured before the timed steps (box_ceiling)
        res["roofline"]["box_ceiling"] = box
        res["roofline"]["frac_vs_box"] = cell_tf / box["mfma_f32_tflops"]
        res["roofline_matvec"]["frac_vs_box"] = kkt_gbs / box["hbm_gbs"]
        per_inst = cell_flop / B * T  # cell flop of one instance's K iterations
        per_gpu = res["value"] / world
        res["step_efficiency"] = {
            "ceiling_spec": FP32_MFMA_PEAK_TFLOPS * 1e12 / per_inst,
            "ceiling_box": box["mfma_f32_tflops"] * 1e12 / per_inst,
            "vs_spec": per_gpu / (FP32_MFMA_PEAK_TFLOPS * 1e12 / per_inst),
            "vs_box": per_gpu / (box["mfma_f32_tflops"] * 1e12 / per_inst),
            "note": "QP instances/s per GPU against the cell GEMM's ceiling (its flop at the fp32 MFMA spec "
                    "peak, and at this box's measured MFMA rate)"}
        res["ranks"] = ranks
        res["ranks_tile_batch"] = parallel.check_tiling(ranks, world * B)
        if st2 is not None:
            st2["roofline"]["frac_vs_box"] = st2["roofline"]["achieved"] / box["mfma_f32_tflops"]
            res["stage2"] = st2
        if trn is not None:
            trn["roofline"]["frac_vs_box"] = trn["roofline"]["achieved"] / box["mfma_f32_tflops"]
            res["train"] = trn
        elif args.train_batch > 0:
            res["train"] = {"skipped": f"one micro-batch of {mb_t} saves {act_bytes / 1e9:.0f} GB of activations "
                                       "over the window (> 70 % of HBM)"}
        if alt is not None:
            res["alt_precision"] = alt
        if rand is not None:
            pr_r, du_r = float(rand[1]["primal"].mean()), float(rand[1]["dual"].mean())
            res["final_residual_random_init"] = {"primal_mean": pr_r, "dual_mean": du_r, "sum": pr_r + du_r}
        if args.cpu_sample > 0 and world == 1:  # the CPU baseline is an N=1 figure
            extra = [("random-init", rand[0], rand[1])] if rand is not None else []
            res["cpu_baseline"] = cpu_baseline(args, d if keep else master, params, out, weights_tag, extra)
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
