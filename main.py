"""Reference-compatible CLI (main.py / configs/QP.yaml of NetSysOpt/I-ADMM-LSTM), HIP-backed.

Same flag names and YAML config as the reference (main.py:22-62; ``-c/--config`` YAML whose
unknown keys are ignored like ``parse_known_args``), plus ``--weight_decay`` which the reference
reads but never registers (main.py:191).  Implemented modes:

  --test   the test loop of main.py:549-1268: load instances (./datasets/QP_{n}_{ineq}_{eq}/
           qp_{id}.gz and the other prob_type layouts of iadmm/dataset.py, the reference's
           gz-pickled dicts, or
           ``--synthetic`` instances from the generate_data.py:67-76 distribution), Ruiz-scale,
           ``test_outer_T`` Stage-I iterations, unscale, per-iteration report on unscaled data,
           "Parallel Time" and the optional ``--save_sol`` .mat file.  All compute runs in
           libiadmm.so kernels (iadmm/solver.py); per-iteration metrics stay on the device and
           are copied once per batch.
  (train)  the training loop of main.py:187-547 for prob_type QP: Ruiz-scaled batches, TBPTT
           windows through the HIP forward/backward kernels (iadmm/train.py), Adam, validation by
           a full no-grad unroll, EarlyStopping checkpoints in the reference's .pth format.
           One process per GPU under torch.distributed.run: each rank trains on its shard of
           every batch and the gradients are all-reduced over RCCL (exact: the loss is a mean).
"""
import argparse
import os
import random
import sys
import time

import numpy as np
import torch
import yaml

import iadmm_path  # noqa: F401
from iadmm import data as qpdata
from iadmm import dataset, ops, solver


def build_parser():
    p = argparse.ArgumentParser(description="train")
    p.add_argument("-c", "--config", type=str)
    add = p.add_argument
    add("--num_var", type=int); add("--num_eq", type=int); add("--num_ineq", type=int)
    add("--prob_type", type=str); add("--qplib_num", type=int)
    add("--scaling_ites", type=int, default=10); add("--input_dim", type=int, default=2)
    add("--hidden_dim", type=int); add("--model_name", type=str); add("--num_layer", type=int)
    add("--sigma", type=float)
    add("--eq_tol", type=float); add("--ineq_tol", type=float); add("--truncated_length", type=int)
    add("--val_frac", type=float); add("--test_frac", type=float); add("--batch_size", type=int)
    add("--device", type=str); add("--lr", type=float); add("--num_epoch", type=int)
    add("--outer_T", type=int); add("--early_stop_mode", type=str)
    add("--patience", type=int, default=100); add("--save_dir", type=str, default="./results/")
    add("--save_sol", action="store_true"); add("--seed", type=int, default=17)
    add("--scaling", action="store_true"); add("--test", action="store_true")
    add("--test_outer_T", type=int); add("--test_batch_size", type=int); add("--data_size", type=int)
    add("--feas_rest", action="store_true"); add("--feas_rest_num", type=int)
    add("--weight_decay", type=float, default=0.0)
    # build-only conveniences
    add("--synthetic", action="store_true", help="generate instances instead of reading ./datasets")
    add("--random_init", action="store_true", help="random-init weights when no checkpoint exists")
    add("--data_dir", type=str, default="./datasets")
    add("--micro_batch", type=int, default=0, help="instances per forward/backward pass (memory)")
    add("--max_minutes", type=float, default=0.0, help="train: stop after the epoch that exceeds this wall time")
    add("--resume", type=str, default="", help="train: state file (model, Adam, epoch, EarlyStopping) written after "
                                               "every epoch and continued from when it exists")
    return p


def parse_args(argv=None):
    """configargparse semantics: YAML supplies defaults, command-line flags win, unknown keys
    (YAML or CLI) are ignored (main.py:22-23, 65)."""
    p = build_parser()
    pre, _ = p.parse_known_args(argv)
    if pre.config:
        with open(pre.config) as f:
            cfg = yaml.safe_load(f) or {}
        known = {a.dest for a in p._actions}
        p.set_defaults(**{k: v for k, v in cfg.items() if k in known})
    args, _ = p.parse_known_args(argv)
    return args


def split_ids(args):
    """main.py:171-183."""
    random.seed(args.seed)
    train_size = int(args.data_size * (1 - args.val_frac - args.test_frac))
    val_size = int(args.data_size * args.val_frac)
    ids = list(range(args.data_size))
    random.shuffle(ids)
    return ids[:train_size], ids[train_size:train_size + val_size], ids[train_size + val_size:]


def load_qp_instances(args, ids, device):
    """Reference on-disk format (main.py:621-722, iadmm/dataset.py): one gzip-pickled dict per
    instance, Q doubled; G/c, A/b optional."""
    path = dataset.instance_dir(args.data_dir, args.num_var, args.num_ineq, args.num_eq, args.prob_type,
                                args.qplib_num)
    d = dataset.read_qp(path, ids, device, args.prob_type, args.qplib_num)
    n, m = d["Q"].shape[1], d["A0"].shape[1]
    mi = d["G"].shape[1] if "G" in d else 0
    me = d["A"].shape[1] if "A" in d else 0
    if mi + me != m:
        raise SystemExit(f"{path}: A0 has {m} rows but G/A give {mi}+{me}; rows outside [G; A] are not supported")
    if (args.num_var, args.num_ineq, args.num_eq) != (n, mi, me):  # sizes come from the data (main.py:656-690)
        args.num_var, args.num_ineq, args.num_eq = n, mi, me
    return d


def checkpoint_path(args, model_name="lstm"):
    """main.py:78-165 save paths (test side main.py:557-612 reads QP_{n}_{eq}_{ineq}_...)."""
    pt, T, h = args.prob_type, args.outer_T, args.hidden_dim
    if pt in ("QP", "QP_RHS"):
        name = f"{pt}_{args.num_var}_{args.num_eq}_{args.num_ineq}_{T}_{h}.pth"
    elif pt in ("Random_QP", "SVM"):
        name = f"{pt}_{args.num_var}_{args.num_ineq}_{T}_{h}.pth"
    elif pt == "Equality_QP":
        name = f"{pt}_{args.num_var}_{args.num_eq}_{T}_{h}.pth"
    elif pt == "QPLIB":
        name = f"{pt}_{args.qplib_num}_{T}_{h}.pth"
    else:
        name = f"{pt}_{T}_{h}.pth"
    return os.path.join(args.save_dir, model_name, "params", name)


def run_test(args):
    from models.lstm import LSTM
    if args.prob_type not in dataset.LAYOUTS or (args.synthetic and args.prob_type != "QP"):
        raise SystemExit(f"prob_type {args.prob_type!r}: datasets of {sorted(dataset.LAYOUTS)}; --synthetic is QP only")
    device = args.device or "cuda:0"
    torch.cuda.set_device(torch.device(device))
    _, _, test_ids = split_ids(args)
    tb = args.test_batch_size
    nb = len(test_ids) // tb
    if args.synthetic:
        allq = None
    else:  # load first: the sizes of non-QP types come from the data
        allq = load_qp_instances(args, test_ids[:nb * tb], device)
    mi, me, n = args.num_ineq, args.num_eq, args.num_var
    model = LSTM(mi + me, args.input_dim, args.hidden_dim, args.outer_T, device)
    ck = checkpoint_path(args, model.name())
    if os.path.exists(ck):
        model.load_state_dict(torch.load(ck, map_location=device, weights_only=True))
    elif not args.random_init:
        raise SystemExit(f"no checkpoint at {ck} (pass --random_init to run with random weights)")
    model.eval()
    T = args.test_outer_T
    packed = solver.PackedWeights()
    reports, total_time, last = [], 0.0, None
    with torch.no_grad():
        if args.synthetic:
            allq = qpdata.make_qp_batch(n, mi, me, nb * tb, first_index=0, seed=args.seed, device=device)
            allq.update(G=allq["A0"][:, :mi], A=allq["A0"][:, mi:], c=allq["zu"][:, :mi], b=allq["zu"][:, mi:])
        for bi in range(nb):
            sl = slice(bi * tb, (bi + 1) * tb)
            d = {k: v[sl].contiguous() for k, v in allq.items()}
            G, A = d.get("G"), d.get("A")
            c = d["c"].reshape(tb, -1) if mi else None
            b = d["b"].reshape(tb, -1) if me else None
            viol = torch.zeros(4, T, tb, device=device)

            def hook(t, x, y, z):  # main.py:959-968, kept on the device
                if mi:
                    iv = ops.bmv(G, x, c, ops.BMV_POS_EXCESS)
                    viol[0, t], viol[1, t] = iv.max(1).values, iv.mean(1)
                if me:
                    ev = ops.bmv(A, x, b, ops.BMV_ABS_GAP)
                    viol[2, t], viol[3, t] = ev.max(1).values, ev.mean(1)

            timer = solver.Timer(True)
            out = solver.solve(model, d["Q"], d["p"], d["A0"], d["zl"], d["zu"], mi, me, T, args.sigma,
                               scaling=args.scaling, scaling_iters=args.scaling_ites, history=True,
                               packed=packed, timer=timer, iter_hook=hook)
            spans = timer.totals_ms()
            total_time += timed_seconds(spans)
            h = {k: out["hist_" + k].mean(1).cpu().numpy() for k in ("obj", "ls_res", "primal", "dual")}
            h["viol"] = viol.mean(2).cpu().numpy()
            if args.feas_rest:  # Stage II on the unscaled data with the last rho (main.py:1035-1066)
                F = args.feas_rest_num
                fvio = torch.zeros(4, F, tb, device=device)

                def fhook(t, x, y, z, sl):  # sl: the Stage-II chunk of the batch
                    if mi:
                        iv = ops.bmv(G[sl].contiguous(), x, c[sl].contiguous(), ops.BMV_POS_EXCESS)
                        fvio[0, t, sl], fvio[1, t, sl] = iv.max(1).values, iv.mean(1)
                    if me:
                        ev = ops.bmv(A[sl].contiguous(), x, b[sl].contiguous(), ops.BMV_ABS_GAP)
                        fvio[2, t, sl], fvio[3, t, sl] = ev.max(1).values, ev.mean(1)

                ftimer = solver.Timer(True)
                rho_rows = solver.rho_rows_of(out["scal"], tb, mi + me, mi)
                s2 = solver.stage2(d["Q"], d["p"].reshape(tb, -1).contiguous(), d["A0"], d["zl"].reshape(tb, -1).contiguous(),
                                   d["zu"].reshape(tb, -1).contiguous(), rho_rows, out["x"].reshape(tb, -1).contiguous(),
                                   out["y"].reshape(tb, -1).contiguous(), out["z"].reshape(tb, -1).contiguous(),
                                   args.sigma, F, timer=ftimer, iter_hook=fhook, history=True)
                total_time += timed_seconds(ftimer.totals_ms())
                for k in ("obj", "ls_res", "primal", "dual"):
                    h["fr_" + k] = s2["hist_" + k].mean(1).cpu().numpy()
                h["fr_viol"] = fvio.mean(2).cpu().numpy()
                out["x"] = s2["x"].unsqueeze(-1)
            reports.append(h)
            last = out
    mean = lambda k: np.mean([r[k] for r in reports], axis=0)  # noqa: E731
    obj, pr, du, vi = mean("obj"), mean("primal"), mean("dual"), mean("viol")
    for t in range(T):  # main.py:1117-1138
        print("Epoch : {} | Test_Obj : {:.3f}".format(t, obj[t]))
        print("Primal_Residuals : {} | Dual_Residuals : {}".format(pr[t], du[t]))
        if mi:
            print("Test_Max_Ineq : {:.3f} | Test_Mean_Ineq : {:.3f} |".format(vi[0, t], vi[1, t]))
        if me:
            print("Test_Max_Eq : {:.3f} | Test_Mean_Eq : {:.3f} |".format(vi[2, t], vi[3, t]))
    if args.feas_rest:  # main.py:1140-1161
        print("-----Starting Sage II-----")
        fr = mean("fr_obj")
        fv = np.mean([r["fr_viol"] for r in reports], axis=0)
        for t in range(args.feas_rest_num):
            print("Epoch : {} | Test_Obj : {:.3f}".format(t, fr[t]))
            if mi:
                print("Test_Max_Ineq : {:.3f} | Test_Mean_Ineq : {:.3f} |".format(fv[0, t], fv[1, t]))
            if me:
                print("Test_Max_Eq : {:.3f} | Test_Mean_Eq : {:.3f} |".format(fv[2, t], fv[3, t]))
    print("Parallel Time : {}".format(total_time / (nb * tb)))
    if args.save_sol:  # main.py:1172-1178, 1248-1268
        import scipy.io as sio
        path = os.path.join(args.save_dir, "lstm", "QP_{}_{}_{}_{}_{}_results.mat".format(
            args.num_var, args.num_eq, args.num_ineq, args.outer_T, args.hidden_dim))
        os.makedirs(os.path.dirname(path), exist_ok=True)
        sio.savemat(path, results_dict(args, total_time, last["x"].cpu().numpy(), reports))
    return reports, total_time


def timed_seconds(spans):
    """Parallel Time of one batch: the solver's timed spans (scaling, iterations, unscale, Stage II
    factor + iterations = the reference's timed model()/exact_model() calls, main.py:881-890,
    1055-1066) without the per-kernel ("k:"), per-iteration metric ("hist:") and untimed
    ("untimed:": the state zero-fills, which the reference allocates before start_time,
    main.py:836-841, and the final residual pass) spans."""
    return sum(v for k, v in spans.items() if not k.startswith(UNTIMED_PREFIXES)) / 1e3


UNTIMED_PREFIXES = ("k:", "hist:", "untimed:")


COND_KEYS = ("x_cond_1_left", "x_cond_1_right", "x_cond_2_left", "x_cond_2_right", "z_cond_1_left",
             "z_cond_1_right", "z_cond_2_left", "z_cond_2_right", "alpha_cond_left", "alpha_cond_right")


def results_dict(args, total_time, x, reports):
    """The --save_sol .mat content with the reference's key set and array shapes
    (main.py:1226-1264):
      objs / ls_res / primal_res / dual_res   [batches, T]  per-batch means per iteration;
      *_fr (Stage II)  main.py:1099-1115 append each batch's list once per Stage-II iteration, so
        objs_fr / primal_res_fr / dual_res_fr are [batches * F, F] (each batch's row F times),
        while ls_res_fr is re-bound per batch (main.py:1052) and holds the last batch's [F];
      *_cond_*  theoretical-condition lists whose computation is commented out in the reference
        (main.py:903-944): one empty list per batch -> [batches, 0]."""
    nb = len(reports)
    d = {"time": total_time, "x": x,
         "objs": np.array([r["obj"] for r in reports]),
         "ls_res": np.array([r["ls_res"] for r in reports]),
         "primal_res": np.array([r["primal"] for r in reports]),
         "dual_res": np.array([r["dual"] for r in reports])}
    if args.feas_rest:
        F = args.feas_rest_num
        rep = lambda k: np.array([r[k] for r in reports for _ in range(F)])  # noqa: E731
        d.update(objs_fr=rep("fr_obj"), ls_res_fr=np.array(reports[-1]["fr_ls_res"]),
                 primal_res_fr=rep("fr_primal"), dual_res_fr=rep("fr_dual"))
    for k in COND_KEYS:
        d[k] = np.zeros((nb, 0))
    return d


_SYNTH_CACHE = {}            # (n, mi, me, seed, device, i) -> one generated instance (on the device)
_SYNTH_CACHE_BYTES = [0]
SYNTH_CACHE_LIMIT = 48 << 30  # device bytes of generated instances kept across epochs


def _synthetic_instance(n, mi, me, i, seed, device):
    """One synthetic instance, generated once and reused by every later epoch (r06: regenerating the
    recipe's 1000 instances -- an fp64 SPD solve each -- took ~13 of the ~70 s of a batch-2 epoch).
    The generator is deterministic per (seed, index), so a cached instance is the one it would make."""
    key = (n, mi, me, seed, str(device), i)
    q = _SYNTH_CACHE.get(key)
    if q is None:
        q = qpdata.make_qp_batch(n, mi, me, 1, first_index=i, seed=seed, device=device)
        nbytes = sum(v.numel() * v.element_size() for v in q.values())
        if _SYNTH_CACHE_BYTES[0] + nbytes <= SYNTH_CACHE_LIMIT:
            _SYNTH_CACHE[key] = q
            _SYNTH_CACHE_BYTES[0] += nbytes
    return q


def _instances(args, ids, device):
    mi, me, n = args.num_ineq, args.num_eq, args.num_var
    if args.synthetic:
        parts = [_synthetic_instance(n, mi, me, i, args.seed, device) for i in ids]
        d = {k: torch.cat([q[k] for q in parts]) for k in parts[0]}
        d.update(G=d["A0"][:, :mi], A=d["A0"][:, mi:], c=d["zu"][:, :mi], b=d["zu"][:, mi:])
        return d
    return load_qp_instances(args, ids, device)


def report_stats(d, x, mi, me, dist):
    """Objective and constraint violations of an unscaled iterate x [B,n] (main.py:367-379,
    497-516): obj mean, ineq/eq violation max-per-instance mean and elementwise mean.  With
    ``dist`` the sums and their counts (instances, elements) are all-reduced over ranks and then
    divided, so unequal shards (parallel.shard differs by one instance) give the global-batch
    means exactly."""
    B = x.shape[0]
    obj, _, _ = ops.metrics(d["Q"], d["p"].reshape(B, -1).contiguous(), d["A0"], x,
                            torch.zeros(B, d["A0"].shape[1], device=x.device),
                            torch.zeros(B, d["A0"].shape[1], device=x.device))
    sums, counts = [obj.double().sum()], [B]
    if mi:
        iv = ops.bmv(d["G"].contiguous(), x, d["c"].reshape(B, -1).contiguous(), ops.BMV_POS_EXCESS)
        sums += [iv.max(1).values.double().sum(), iv.double().sum()]
        counts += [B, iv.numel()]
    if me:
        ev = ops.bmv(d["A"].contiguous(), x, d["b"].reshape(B, -1).contiguous(), ops.BMV_ABS_GAP)
        sums += [ev.max(1).values.double().sum(), ev.double().sum()]
        counts += [B, ev.numel()]
    t = torch.cat([torch.stack(sums), torch.tensor(counts, dtype=torch.float64, device=x.device)])
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    k = len(sums)
    t = (t[:k] / t[k:]).tolist()
    out = {"obj": t.pop(0)}
    if mi:
        out["ineq_max"], out["ineq_mean"] = t.pop(0), t.pop(0)
    if me:
        out["eq_max"], out["eq_mean"] = t.pop(0), t.pop(0)
    return out


def save_resume_state(path, model, optimizer, epoch, stopper):
    """The --resume state file: tensors and plain Python scalars only, so that
    torch.load(weights_only=True) reads it back (EarlyStopping's best_loss becomes an np.float64
    after its second improvement, utils.py:40, which the weights-only unpickler refuses).  Written
    to a temporary file and renamed into place, so a run killed mid-write keeps the previous state."""
    best = stopper.best_loss
    state = {"model": model.state_dict(), "optimizer": optimizer.state_dict(), "epoch": int(epoch),
             "best_loss": None if best is None else float(best), "counter": int(stopper.counter)}
    tmp = path + ".tmp"
    torch.save(state, tmp)
    os.replace(tmp, path)


def run_train(args):
    """main.py:187-547 (QP): epochs of TBPTT batches + validation + EarlyStopping."""
    from iadmm import parallel, train
    from models.lstm import LSTM
    from utils import EarlyStopping
    if args.prob_type != "QP":
        raise SystemExit(f"prob_type {args.prob_type!r} is out of scope (DESIGN.md §0); use QP")
    world, rank, local = parallel.env()
    device = f"cuda:{local}" if world > 1 else (args.device or "cuda:0")
    torch.cuda.set_device(torch.device(device))
    dist = parallel.init("nccl", local) if world > 1 else None
    mi, me = args.num_ineq, args.num_eq
    torch.manual_seed(args.seed)
    model = LSTM(mi + me, args.input_dim, args.hidden_dim, args.outer_T, device)
    save_path = os.path.join(args.save_dir, model.name(), "params", "QP_{}_{}_{}_{}_{}.pth".format(
        args.num_var, args.num_ineq, args.num_eq, args.outer_T, args.hidden_dim))  # main.py:88-92
    if rank == 0:
        os.makedirs(os.path.dirname(save_path), exist_ok=True)
    stopper = EarlyStopping(save_path, patience=args.patience)
    optimizer = torch.optim.Adam(model.parameters(), lr=args.lr, weight_decay=args.weight_decay)
    train_ids, val_ids, _ = split_ids(args)
    packed = solver.PackedWeights()
    history = []
    t_start = time.time()
    first_epoch = 0
    if args.resume and os.path.exists(args.resume):  # this repo's own state file (tensors + scalars only)
        st = torch.load(args.resume, map_location=device, weights_only=True)
        model.load_state_dict(st["model"])
        optimizer.load_state_dict(st["optimizer"])
        stopper.best_loss, stopper.counter = st["best_loss"], int(st["counter"])
        first_epoch = int(st["epoch"]) + 1
        if rank == 0:
            print(f"[train] resumed from {args.resume} after epoch {first_epoch - 1}", file=sys.stderr, flush=True)
    for epoch in range(first_epoch, args.num_epoch):
        model.train()
        t0 = time.time()
        loss = float("nan")
        last = {}
        n_batches = int(len(train_ids) / args.batch_size)
        for bi in range(n_batches):
            ids = train_ids[bi * args.batch_size:(bi + 1) * args.batch_size]
            first, count = parallel.shard(len(ids), world, rank)
            d = _instances(args, ids[first:first + count], device)
            Dsc = None
            if args.scaling:
                sc = ops.ruiz_scale(d["Q"], d["p"], d["A0"], d["zl"], d["zu"], args.scaling_ites)
                ds, Dsc = dict(zip(("Q", "p", "A0", "zl", "zu"), sc[:5])), sc[5]
                del sc
            else:
                ds = d
            fin = {}
            loss = train.tbptt_batch(model, ds, mi, me, args.outer_T, args.truncated_length, args.sigma, optimizer,
                                     micro_batch=args.micro_batch or None, global_batch=len(ids), dist=dist,
                                     final=fin)
            if bi == n_batches - 1:  # only the epoch's last batch is reported (main.py:362-379)
                last = dict(d=d, x=fin["x"].reshape(count, -1) * (Dsc.reshape(count, -1) if Dsc is not None else 1.0))
            del d, ds, fin
            if rank == 0 and (bi + 1) % 50 == 0:
                print(f"[train] epoch {epoch} batch {bi + 1}/{n_batches} loss {loss:.4f} "
                      f"{time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        train_time = time.time() - t0
        # main.py:362-379: objective and violations of the last training batch's final iterate
        # (unscaled); each rank holds its shard, so the means are combined over ranks
        tr = report_stats(last["d"], last["x"].contiguous(), mi, me, dist) if last else None
        # validation: full unroll under no_grad (main.py:382-510), metrics on unscaled x
        model.eval()
        t0 = time.time()
        with torch.no_grad():
            v = _instances(args, val_ids, device)
            out = solver.solve(model, v["Q"], v["p"], v["A0"], v["zl"], v["zu"], mi, me, args.outer_T, args.sigma,
                               scaling=args.scaling, scaling_iters=args.scaling_ites, packed=packed)
            va = report_stats(v, out["x"].reshape(len(val_ids), -1).contiguous(), mi, me, None)
            val_obj = va["obj"]
            vios = ([va["ineq_max"]] if mi else []) + ([va["eq_max"]] if me else [])
        val_time = time.time() - t0
        stop = False
        if rank == 0:
            stop = stopper.step(val_obj, model, args.early_stop_mode or "min", args.eq_tol, *vios)
            if args.max_minutes and time.time() - t_start > 60.0 * args.max_minutes:
                stop = True  # decided on rank 0 and broadcast below, like the early stop
            tobj = tr["obj"] if tr else float("nan")
            print("Epoch : {} | Train_Obj : {:.3f} | Val_Obj : {:.3f} | Train_Time : {:.3f} | Val_Time : {:.3f} |".format(
                epoch, tobj, val_obj, train_time, val_time), flush=True)
            for key, name, on in (("ineq", "Ineq", mi), ("eq", "Eq", me)):
                if on and tr:  # main.py:537-541
                    print("Epoch : {} | Train_Max_{} : {:.3f} | Train_Mean_{} : {:.3f} | Val_Max_{} : {:.3f} | "
                          "Val_Mean_{} : {:.3f} |".format(epoch, name, tr[key + "_max"], name, tr[key + "_mean"],
                                                          name, va[key + "_max"], name, va[key + "_mean"]), flush=True)
        if dist is not None:
            flag = torch.tensor([1 if stop else 0], device=device)
            dist.broadcast(flag, 0)
            stop = bool(flag.item())
        history.append((loss, val_obj))
        if args.resume and rank == 0:
            save_resume_state(args.resume, model, optimizer, epoch, stopper)
        if stop:
            break
    if dist is not None:
        dist.destroy_process_group()
    return history


def main(argv=None):
    args = parse_args(argv)
    if args.test:
        return run_test(args)
    return run_train(args)


if __name__ == "__main__":
    main(sys.argv[1:])
