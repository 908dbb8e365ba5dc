"""End-to-end CLI (main.py --test) on the GPU: reference command line, synthetic instances,
random-init weights; the per-iteration report and the .mat writer work and the final residuals
equal the solver's."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_main_test_mode(tmp_path, capsys):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import main
    cfg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "QP.yaml")
    argv = ["--config", cfg, "--prob_type", "QP", "--num_var", "60", "--num_ineq", "20", "--num_eq", "10",
            "--outer_T", "8", "--hidden_dim", "40", "--scaling", "--test", "--test_outer_T", "8",
            "--test_batch_size", "4", "--data_size", "100", "--test_frac", "0.1", "--val_frac", "0.1",
            "--save_sol", "--save_dir", str(tmp_path), "--synthetic", "--random_init", "--feas_rest",
            "--feas_rest_num", "3"]
    reports, total = main.main(argv)
    out = capsys.readouterr().out
    assert out.count("Primal_Residuals") == 8 and "Parallel Time" in out
    assert "Test_Max_Ineq" in out and "Test_Max_Eq" in out
    assert "Starting Sage II" in out and out.count("Test_Obj") == 8 + 3
    assert len(reports) == 2 and total > 0
    import scipy.io as sio
    mat = sio.loadmat(os.path.join(tmp_path, "lstm", "QP_60_10_20_8_40_results.mat"))
    assert mat["primal_res"].shape == (2, 8)
    assert np.isfinite(mat["dual_res"]).all()
    # the reference's key set and shapes with --feas_rest (main.py:1226-1245)
    ref_keys = {"time", "x", "objs", "ls_res", "primal_res", "dual_res", "objs_fr", "ls_res_fr", "primal_res_fr",
                "dual_res_fr"} | set(main.COND_KEYS)
    assert {k for k in mat if not k.startswith("__")} == ref_keys
    assert mat["objs_fr"].shape == (2 * 3, 3) and mat["primal_res_fr"].shape == (2 * 3, 3)
    assert mat["ls_res_fr"].shape == (1, 3) and mat["x_cond_1_left"].shape == (2, 0)
    assert np.allclose(mat["objs_fr"][0], mat["objs_fr"][2]) and np.isfinite(mat["dual_res_fr"]).all()
    # Stage II solves K xv = b~ exactly: its linear-system residual is round-off level
    assert (mat["ls_res_fr"] < 1e-2 * np.abs(mat["ls_res"]).max()).all()


def test_main_train_mode_improves_loss(tmp_path, capsys):
    """main.py training mode (synthetic QPs): the TBPTT loss goes down over a few epochs and the
    EarlyStopping checkpoint is written in the reference's .pth format."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import main
    argv = ["--prob_type", "QP", "--num_var", "40", "--num_ineq", "16", "--num_eq", "8", "--outer_T", "10",
            "--truncated_length", "5", "--hidden_dim", "32", "--sigma", "6e-6", "--scaling", "--lr", "0.002",
            "--batch_size", "4", "--data_size", "40", "--val_frac", "0.1", "--test_frac", "0.1",
            "--num_epoch", "4", "--eq_tol", "1e9", "--ineq_tol", "1e9", "--early_stop_mode", "min",
            "--save_dir", str(tmp_path), "--synthetic", "--micro_batch", "2", "--patience", "10"]
    hist = main.main(argv)
    assert len(hist) == 4
    out = capsys.readouterr().out
    # the reference's epoch report (main.py:537-541)
    assert out.count("| Train_Obj : ") == 4 and out.count("| Val_Obj : ") == 4
    assert out.count("| Train_Max_Ineq : ") == 4 and out.count("| Val_Mean_Ineq : ") == 4
    assert out.count("| Train_Max_Eq : ") == 4 and out.count("| Val_Mean_Eq : ") == 4
    assert hist[-1][0] < hist[0][0]
    sd = torch.load(os.path.join(tmp_path, "lstm", "params", "QP_40_16_8_10_32.pth"), weights_only=True)
    assert set(sd) >= {"W_i", "U_u", "W_h", "b_h", "rho", "alpha"}
