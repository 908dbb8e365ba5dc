"""On-disk instance format (row f3): the reference's gz-pickled dicts (generate_data.py:85-92)
read back the way main.py:621-722 loads them."""
import gzip
import os
import pickle

import numpy as np
import pytest
import torch

from iadmm import data, dataset


def _reference_style_files(tmp, n, mi, me, count, seed=0):
    """Files laid out exactly as generate_data.py:67-92 writes them (numpy fp64, Q = 0.5 diag)."""
    rng = np.random.default_rng(seed)
    recs = []
    for i in range(count):
        Q0 = 0.5 * np.diag(rng.random(n))
        p0 = rng.random((n, 1))
        A = rng.normal(size=(me, n))
        b = 2 * rng.random((me, 1)) - 1
        G = rng.normal(size=(mi, n))
        c = np.sum(np.abs(G @ np.linalg.pinv(A)), axis=1).reshape(mi, 1)
        rec = {"Q": Q0, "p": p0, "G": G, "c": c, "A": A, "b": b, "A0": np.concatenate((G, A)),
               "zl": np.concatenate((-np.inf * np.ones(c.shape), b)), "zu": np.concatenate((c, b)),
               "x": rng.random(n), "y": rng.random(mi + me)}
        with gzip.open(os.path.join(tmp, f"qp_{i}.gz"), "wb") as f:
            pickle.dump(rec, f)
        recs.append(rec)
    return recs


def test_reads_reference_layout(tmp_path):
    n, mi, me = 10, 4, 3
    recs = _reference_style_files(str(tmp_path), n, mi, me, 5)
    ids = [3, 0, 4]
    d = dataset.read_qp(str(tmp_path), ids, "cpu")
    # the reference's own conversion: torch.tensor(np.array(list), float32) (* 2 for Q)
    ref = lambda k: torch.tensor(np.array([recs[i][k] for i in ids]), dtype=torch.float32)  # noqa: E731
    assert torch.equal(d["Q"], ref("Q") * 2)
    for k in ("p", "A0", "zl", "zu", "G", "c", "A", "b"):
        assert torch.equal(d[k], ref(k)), k
    assert d["p"].shape == (3, n, 1) and d["zl"].shape == (3, mi + me, 1)
    assert torch.isinf(d["zl"][:, :mi]).all()
    assert "lb" not in d


def test_write_read_round_trip(tmp_path):
    n, mi, me = 16, 6, 4
    d = data.make_qp_batch(n, mi, me, 3, first_index=5, device="cpu")
    out = dataset.instance_dir(str(tmp_path), n, mi, me)
    dataset.write_qp(out, d, mi, first_index=5)
    assert sorted(os.listdir(out)) == ["qp_5.gz", "qp_6.gz", "qp_7.gz"]
    r = dataset.read_qp(out, [5, 6, 7], "cpu")
    for k in ("Q", "p", "A0", "zl", "zu"):
        assert torch.equal(r[k], d[k]), k
    assert torch.equal(r["G"], d["A0"][:, :mi]) and torch.equal(r["b"], d["zu"][:, mi:])


def test_equality_only_and_sparse(tmp_path):
    sp = pytest.importorskip("scipy.sparse")
    n, me = 8, 5
    rng = np.random.default_rng(1)
    A = rng.normal(size=(me, n))
    b = rng.random((me, 1))
    rec = {"Q": sp.csr_matrix(np.diag(rng.random(n))), "p": sp.csr_matrix(rng.random((n, 1))),
           "A": sp.csr_matrix(A), "b": sp.csr_matrix(b), "A0": sp.csr_matrix(A),
           "zl": sp.csr_matrix(b), "zu": sp.csr_matrix(b)}
    out = dataset.instance_dir(str(tmp_path), n, 0, me, "Equality_QP")
    os.makedirs(out)
    with gzip.open(dataset.instance_file(out, 0, "Equality_QP"), "wb") as f:
        pickle.dump(rec, f)
    d = dataset.read_qp(out, [0], "cpu", "Equality_QP")
    assert "G" not in d and d["A"].shape == (1, me, n)
    assert torch.equal(d["Q"][0], torch.tensor(rec["Q"].toarray(), dtype=torch.float32) * 2)


def test_errors(tmp_path):
    with pytest.raises(FileNotFoundError):
        dataset.read_qp(str(tmp_path), [0], "cpu")
    with pytest.raises(ValueError):
        dataset.instance_dir(str(tmp_path), 1, 1, 1, "NotAType")
    with gzip.open(os.path.join(str(tmp_path), "qp_0.gz"), "wb") as f:
        pickle.dump({"Q": np.eye(2)}, f)
    with pytest.raises(KeyError):
        dataset.read_qp(str(tmp_path), [0], "cpu")


def test_main_loader_infers_sizes(tmp_path):
    import main
    n, mi, me = 12, 5, 3
    out = dataset.instance_dir(str(tmp_path), n, mi, me)
    os.makedirs(out)
    _reference_style_files(out, n, mi, me, 2)
    args = main.parse_args(["--prob_type", "QP", "--num_var", str(n), "--num_ineq", str(mi), "--num_eq", str(me),
                            "--data_dir", str(tmp_path)])
    d = main.load_qp_instances(args, [0, 1], "cpu")
    assert d["A0"].shape == (2, mi + me, n)
    assert main.checkpoint_path(args).endswith(f"QP_{n}_{me}_{mi}_{args.outer_T}_{args.hidden_dim}.pth")


def test_generate_data_cli(tmp_path):
    import generate_data
    generate_data.main(["--prob_type", "QP", "--num_var", "8", "--num_ineq", "3", "--num_eq", "2",
                        "--data_size", "3", "--data_dir", str(tmp_path), "--device", "cpu", "--chunk", "2"])
    out = dataset.instance_dir(str(tmp_path), 8, 3, 2)
    r = dataset.read_qp(out, [0, 1, 2], "cpu")
    ref = data.make_qp_batch(8, 3, 2, 3, device="cpu")
    assert torch.equal(r["A0"], ref["A0"]) and torch.equal(r["zu"], ref["zu"])


def test_threaded_equals_sequential(tmp_path):
    """The thread-pool reader/writer (workers > 1) produce exactly the sequential result."""
    n, mi, me = 24, 7, 5
    d = data.make_qp_batch(n, mi, me, 9, first_index=0, device="cpu")
    seq, par = os.path.join(str(tmp_path), "seq"), os.path.join(str(tmp_path), "par")
    dataset.write_qp(seq, d, mi, workers=1)
    dataset.write_qp(par, d, mi, workers=4)
    ids = [8, 0, 3, 5, 1]
    a = dataset.read_qp(seq, ids, "cpu", workers=1)
    b = dataset.read_qp(par, ids, "cpu", workers=4)
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k
    for k in ("Q", "p", "A0", "zl", "zu"):
        assert torch.equal(a[k], d[k][ids]), k


def test_inconsistent_shapes_raise(tmp_path):
    n, mi, me = 8, 3, 2
    _reference_style_files(str(tmp_path), n, mi, me, 2)
    with gzip.open(os.path.join(str(tmp_path), "qp_1.gz"), "rb") as f:
        rec = pickle.load(f)  # file written by this test
    rec["A0"] = rec["A0"][:, :-1]
    with gzip.open(os.path.join(str(tmp_path), "qp_1.gz"), "wb") as f:
        pickle.dump(rec, f)
    with pytest.raises(ValueError):
        dataset.read_qp(str(tmp_path), [0, 1], "cpu")
