"""Dataset writer with the reference's CLI (generate_data.py:15-27, QP branch :67-92).

  python generate_data.py --prob_type QP --num_var 1000 --num_ineq 500 --num_eq 500 --data_size 1024

writes ./datasets/QP_{n}_{ineq}_{eq}/qp_{i}.gz in the reference's format (iadmm/dataset.py) from the
build's per-instance-seeded generator (iadmm/data.py).  Differences from the reference, stated:
OSQP is not available, so instances are not filtered on OSQP's "solved" status and no 'x'/'y'
solutions are stored; instance i is drawn from its own generator (seed + i), not from one batch draw.
"""
import argparse

import torch

import iadmm_path  # noqa: F401
from iadmm import data, dataset


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("-c", "--config", type=str)
    ap.add_argument("--num_var", type=int, required=True)
    ap.add_argument("--num_eq", type=int, required=True)
    ap.add_argument("--num_ineq", type=int, required=True)
    ap.add_argument("--prob_type", type=str, default="QP")
    ap.add_argument("--data_size", type=int, required=True)
    ap.add_argument("--seed", type=int, default=17)
    ap.add_argument("--data_dir", type=str, default="./datasets")
    ap.add_argument("--chunk", type=int, default=256, help="instances generated per device batch")
    ap.add_argument("--device", type=str, default="cuda" if torch.cuda.is_available() else "cpu")
    args, _ = ap.parse_known_args(argv)
    if args.prob_type != "QP":
        raise SystemExit("only the QP generator (generate_data.py:67-92) is restated")
    out = dataset.instance_dir(args.data_dir, args.num_var, args.num_ineq, args.num_eq)
    for s in range(0, args.data_size, args.chunk):
        b = min(args.chunk, args.data_size - s)
        d = data.make_qp_batch(args.num_var, args.num_ineq, args.num_eq, b, first_index=s, seed=args.seed,
                               device=args.device)
        dataset.write_qp(out, d, args.num_ineq, first_index=s)
    print(f"wrote {args.data_size} instances to {out}")


if __name__ == "__main__":
    main()
