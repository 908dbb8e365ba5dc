"""Host logic of the CLI (main.py) that needs no GPU: which solver spans count as the
reference's "Parallel Time" (main.py:825-834, 881-890, 1024-1031, 1055-1066)."""
import os
import re

import iadmm_path  # noqa: F401
import main

from conftest import PKG

# the reference times Ruiz scaling, the model() calls, the final unscale and Stage II; it does
# not time the zero-fills of the state (allocated before start_time, main.py:836-841) or metrics
TIMED = {"scaling", "setup", "iterations", "unscale", "stage2_assemble", "stage2_factor", "stage2_iterations"}


def _span_names():
    names = set()
    for fn in ("solver.py",):
        src = open(os.path.join(PKG, "iadmm", fn)).read()
        names |= set(re.findall(r'timer\.start\("([^"]+)"\)', src))
    return names


def test_timed_seconds_sums_only_the_reference_timed_spans():
    names = _span_names()
    assert {"scaling", "setup", "iterations", "unscale", "untimed:setup", "untimed:metrics"} <= names
    spans = {k: 1000.0 for k in names}
    spans.update({"k:lstm_cell": 5000.0, "hist:metrics": 7000.0})
    counted = {k for k in spans if main.timed_seconds({k: spans[k]}) > 0}
    assert counted == TIMED & names, counted
    assert main.timed_seconds(spans) == len(TIMED & names)


def test_stage2_chunks_are_balanced():
    """solver.stage2_chunk: equal chunks under the memory cap (config 4: 512 instances whose dense
    K fit 410 at a time run as 256 + 256, not 410 + 102); the whole batch when it fits."""
    from iadmm import solver
    per = lambda N: 4 * N * N + 64 * N  # noqa: E731
    assert solver.stage2_chunk(512, 10000, budget_bytes=410 * per(10000)) == 256
    assert solver.stage2_chunk(1024, 2000, budget_bytes=2000 * per(2000)) == 1024
    assert solver.stage2_chunk(5, 100, budget_bytes=2 * per(100)) == 2
    assert solver.stage2_chunk(7, 100, budget_bytes=3 * per(100)) == 3
    assert solver.stage2_chunk(3, 100, budget_bytes=0) == 1


def test_resume_state_reloads_weights_only_after_np_best_loss(tmp_path):
    """EarlyStopping's best_loss is an np.float64 after its second improvement (utils.py:40, the
    reference's np.min); the --resume state file must still load with weights_only=True, and the
    write goes through a temporary file renamed into place."""
    import numpy as np
    import torch
    from utils import EarlyStopping
    model = torch.nn.Linear(3, 2)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    stopper = EarlyStopping(str(tmp_path / "ck.pth"), patience=5)
    stopper.step(2.0, model, "min", 1.0)
    stopper.step(1.5, model, "min", 1.0)
    assert isinstance(stopper.best_loss, np.floating)
    path = str(tmp_path / "resume.pt")
    main.save_resume_state(path, model, opt, 3, stopper)
    assert not os.path.exists(path + ".tmp")
    st = torch.load(path, weights_only=True)
    assert st["best_loss"] == 1.5 and type(st["best_loss"]) is float
    assert st["epoch"] == 3 and st["counter"] == 0
    stopper.best_loss = None
    main.save_resume_state(path, model, opt, 4, stopper)
    assert torch.load(path, weights_only=True)["best_loss"] is None


def test_synthetic_instances_cached_across_epochs():
    """r06: main.py generates each synthetic instance once and reuses it in later epochs; the cached
    instance is the one the generator makes (deterministic per seed and index), and callers get copies."""
    import argparse
    import torch
    main._SYNTH_CACHE.clear()
    main._SYNTH_CACHE_BYTES[0] = 0
    args = argparse.Namespace(num_ineq=3, num_eq=2, num_var=6, synthetic=True, seed=100017)
    d1 = main._instances(args, [4, 7], "cpu")
    assert len(main._SYNTH_CACHE) == 2 and main._SYNTH_CACHE_BYTES[0] > 0
    d2 = main._instances(args, [7, 4], "cpu")
    assert len(main._SYNTH_CACHE) == 2
    assert torch.equal(d1["Q"][0], d2["Q"][1]) and torch.equal(d1["A0"][1], d2["A0"][0])
    from iadmm import data as qpdata
    ref = qpdata.make_qp_batch(6, 3, 2, 1, first_index=7, seed=100017, device="cpu")
    for k in ("Q", "p", "A0", "zl", "zu"):
        assert torch.equal(d1[k][1:2], ref[k]), k
    d2["Q"].zero_()  # a caller's tensors are not the cache's
    assert torch.equal(main._instances(args, [4], "cpu")["Q"][0], d1["Q"][0])
    main._SYNTH_CACHE.clear()
    main._SYNTH_CACHE_BYTES[0] = 0
