"""CPU-side checks of the C-ABI boundary: the HIP library loads without a GPU and exports every
entry point include/iadmm.h declares, with the argument counts the ctypes layer binds."""
import os
import re

import pytest

import iadmm_path  # noqa: F401
from iadmm import _abi

from conftest import REPO

HEADER = os.path.join(REPO, "include", "iadmm.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return {m.group(1): m.group(2) for m in re.finditer(r"\b(iadmm_\w+)\s*\(([^)]*)\)\s*;", src)}


def test_library_loads_and_exports_header_symbols():
    lib = _abi.lib()
    decl = declared()
    assert len(decl) >= 15
    missing = [name for name in decl if getattr(lib, name, None) is None]
    assert not missing, f"declared in iadmm.h but not exported: {missing}"


def test_ctypes_signatures_match_header_arity():
    for name, args in declared().items():
        assert name in _abi.SIGNATURES, f"{name} not bound in _abi.SIGNATURES"
        n_header = 0 if args.strip() in ("", "void") else len(args.split(","))
        assert len(_abi.SIGNATURES[name][1]) == n_header, name


def test_size_queries_without_gpu():
    lib = _abi.lib()
    assert lib.iadmm_lstm_ntiles(800) == 25
    assert lib.iadmm_lstm_ntiles(40) == 2
    assert lib.iadmm_lstm_packed_floats(800) == 25 * 25 * 128 * 32
    assert lib.iadmm_version() > 0
    # KKT workspace: dots + r (2 (n+m)), one partial column-sum vector per 256-row block and two
    # partial sums per 256-row chunk of [n ; m]
    assert lib.iadmm_kkt_resgrad_ws_bytes(3, 1000, 1000) == 3 * (2 * 2000 + (4 + 4) * 1000 + 2 * 8) * 4
    assert lib.iadmm_kkt_resgrad_ws_bytes(1, 24, 0) == (2 * 24 + 1 * 24 + 2 * 1) * 4
    # LDS of the split sweeps (the IADMM_E_SIZE limit): vectors + 8 fold rows below 64 KiB, 4 above
    assert lib.iadmm_kkt_resgrad_lds_bytes(1000, 1000) == (2000 + 8 * 1000) * 4
    assert lib.iadmm_kkt_resgrad_lds_bytes(5000, 5000) == (10000 + 4 * 2048) * 4
    assert lib.iadmm_kkt_resgrad_lds_bytes(16384, 16384) == 160 * 1024


def lib_lds_over(n, m):
    return _abi.lib().iadmm_kkt_resgrad_lds_bytes(n, m) > 160 * 1024


def test_bad_arguments_rejected_before_launch():
    # argument checks run on the host before any HIP call: safe without a GPU
    with pytest.raises(_abi.IadmmError, match="bad argument"):
        _abi.call("iadmm_kkt_resgrad", 0, 10, 10, 5, *([None] * 7), 1.0, None, None, None, None, None, None, 0,
                  None)
    with pytest.raises(_abi.IadmmError, match="bad argument"):  # workspace missing / too small
        _abi.call("iadmm_kkt_resgrad", 2, 10, 10, 5, *([16] * 7), 1.0, 16, 16, None, None, None, 16, 100, None)
    assert lib_lds_over(20000, 20000)
    with pytest.raises(_abi.IadmmError, match="size beyond"):
        _abi.call("iadmm_kkt_resgrad", 1, 20000, 20000, 0, *([16] * 7), 1.0, 16, 16, None, None, None, 16, 1 << 40,
                  None)
    with pytest.raises(_abi.IadmmError, match="bad argument"):
        _abi.call("iadmm_lstm_cell_fwd", 10, 8, 16, 16, 16, 16, 16, 16, 16, 16, 16, None)


def test_lu_factor_workspace_is_caller_owned():
    """iadmm_lu_factor takes its scratch from the caller (no allocation inside the
    library): the size query answers without a GPU and a missing or short workspace is refused."""
    lib = _abi.lib()
    assert lib.iadmm_lu_factor_ws_bytes(1024, 2000) >= 1024 * (4 * 64 + 1) * 4
    assert lib.iadmm_lu_factor_ws_bytes(0, 2000) == 0
    need = lib.iadmm_lu_factor_ws_bytes(2, 100)
    with pytest.raises(_abi.IadmmError, match="bad argument"):
        _abi.call("iadmm_lu_factor", 2, 100, 16, 16, 16, None, need, None)
    with pytest.raises(_abi.IadmmError, match="bad argument"):
        _abi.call("iadmm_lu_factor", 2, 100, 16, 16, 16, 16, need - 4, None)
    with pytest.raises(_abi.IadmmError, match="misaligned"):
        _abi.call("iadmm_lu_factor", 2, 100, 16, 16, 16, 20, need, None)


def test_lu_size_limit_is_the_hbm_forms():
    """Stage II sizes (r04): above the LDS-resident solve's N = 36736 the HBM forms take over
    (tests/test_lu_hbm_gpu.py runs N = 36800); both entry points refuse only N > 46340 (N * N must
    stay below 2^31), before touching any pointer."""
    lib = _abi.lib()
    need = lib.iadmm_lu_factor_ws_bytes(1, 46341)
    with pytest.raises(_abi.IadmmError, match="size beyond"):
        _abi.call("iadmm_lu_factor", 1, 46341, 16, 16, 16, 16, need, None)
    with pytest.raises(_abi.IadmmError, match="size beyond"):
        _abi.call("iadmm_lu_solve", 1, 46341, 16, 16, 16, None)


def _csrc_without_comments():
    csrc = os.path.join(REPO, "i-admm-lstm_amd", "csrc")
    for fn in sorted(os.listdir(csrc)):
        yield fn, re.sub(r"//[^\n]*|/\*.*?\*/", "", open(os.path.join(csrc, fn)).read(), flags=re.S)


def test_no_device_allocation_inside_the_library():
    """Every device buffer is caller-owned: no hipMalloc* / hipFree* call in the HIP sources."""
    hits = []
    for fn, src in _csrc_without_comments():
        hits += [f"{fn}: {m.group(0)}" for m in re.finditer(r"\bhip(Malloc|Free)\w*", src)]
    assert not hits, hits


def test_no_hidden_state_inside_the_library():
    """include/iadmm.h's contract: the only HIP objects the library creates are
    an iadmm_lu_ctx's streams and events, made and destroyed in iadmm_lu_ctx_create / _destroy; no
    mutex, no function-static or namespace-scope mutable object, no environment read anywhere."""
    hits = []
    for fn, src in _csrc_without_comments():
        for m in re.finditer(r"\bhip(StreamCreate|EventCreate|StreamDestroy|EventDestroy)\w*", src):
            # the enclosing function: the last extern "C" / static definition before the match
            head = src[:m.start()]
            fns = re.findall(r"\b(iadmm_\w+|\w+)\s*\([^;{]*\)\s*\{", head)
            owner = fns[-1] if fns else "?"
            if owner not in ("iadmm_lu_ctx_create", "iadmm_lu_ctx_destroy"):
                hits.append(f"{fn}: {m.group(0)} in {owner}")
        hits += [f"{fn}: {m.group(0)}" for m in re.finditer(r"\bgetenv\b|std::mutex|\bthread_local\b", src)]
        hits += [f"{fn}: static local {m.group(0)!r}" for m in
                 re.finditer(r"\n\s+static\s+(?!constexpr|const\b|inline|__device__|IADMM_DEV|void|int|bool|float)\w[^;(]*;", src)]
    assert not hits, hits


def test_lu_context_abi():
    """The look-ahead context is created / destroyed through its two calls (no GPU needed to check
    the argument handling); a NULL context means "everything on the caller's stream"."""
    lib = _abi.lib()
    assert lib.iadmm_lu_ctx_destroy(None) == 0
    with pytest.raises(_abi.IadmmError, match="bad argument"):
        _abi.call("iadmm_lu_ctx_create", None)
    need = lib.iadmm_lu_factor_ws_bytes(2, 100)
    with pytest.raises(_abi.IadmmError, match="bad argument"):  # unknown flag bits
        _abi.call("iadmm_lu_factor_ex", 2, 100, 16, 16, 16, 16, need, None, 8, None)
    with pytest.raises(_abi.IadmmError, match="bad argument"):
        _abi.call("iadmm_lu_solve_ex", 2, 100, 16, 16, 16, 2, None)


def test_lu_flag_constants_match_header():
    """ops' LU flag constants are the header's enum values (IADMM_LU_PAIRS is the default since r05,
    IADMM_LU_RANK128 selects the r04 rank-128 form)."""
    import re
    from iadmm import ops
    hdr = open(HEADER).read()
    enum = dict((k, int(v)) for k, v in re.findall(r"(IADMM_LU_\w+)\s*=\s*(\d+)", hdr))
    assert enum == {"IADMM_LU_FORCE_HBM": ops.LU_FORCE_HBM, "IADMM_LU_PAIRS": ops.LU_PAIRS,
                    "IADMM_LU_RANK128": ops.LU_RANK128}


def test_lib_path_override_limited_to_variant_dirs(tmp_path):
    """IADMM_LIB_PATH (tools/ variant studies) cannot point the product path at an arbitrary library
    (VERDICT r05 item 9)."""
    import subprocess
    import sys
    bad = tmp_path / "libother.so"
    bad.write_bytes(b"")
    code = "import iadmm_path; from iadmm import _abi"
    env = dict(os.environ, IADMM_LIB_PATH=str(bad))
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, env=env, capture_output=True, text=True)
    assert r.returncode != 0 and "tools/ or variants/" in r.stderr
    env["IADMM_LIB_PATH"] = ""
    r = subprocess.run([sys.executable, "-c", code + "; print(_abi.LIB_PATH)"], cwd=REPO, env=env,
                       capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip().endswith("iadmm/libiadmm.so"), r.stderr


def test_small_m_gemm_split_policy():
    """r06: the split counts of the training GEMMs (iadmm/ops.py) at the recipe's batch 2 and the
    config-5 micro-batch, with the CU count given; the K-part size query is a host function."""
    from iadmm import ops
    lib = _abi.lib()
    assert lib.iadmm_gemm_nt_kpart(3200, 6) == 544 and lib.iadmm_gemm_nt_kpart(3200, 1) == 3200
    assert lib.iadmm_gemm_nt_kpart(48, 3) == 32 and lib.iadmm_gemm_nt_kpart(0, 3) == 0
    saved = dict(ops._CU_COUNT)
    dev = ops.torch.cuda.current_device
    try:
        ops.torch.cuda.current_device = lambda: 0
        ops._CU_COUNT[0] = 256
        # batch 2 (M = 4000 rows): one round of 512 workgroup slots
        assert ops.gemm_nt_ksplit(4000, 800, 3200) == 6          # 80 tiles x 6 = 480
        assert ops.gemm_tn_rows_per_split(4000, 800, 3200) == 576  # 65 tiles x 7 slices = 455
        assert ops.gemm_tn_rows_per_split(4000, 3, 3200) == 32
        # config-5 micro-batch (M = 256000): the r01-r05 splits, bitwise-unchanged gradients
        assert ops.gemm_nt_ksplit(256000, 800, 3200) == 1
        assert ops.gemm_tn_rows_per_split(256000, 800, 3200) == 4096
        assert ops.gemm_tn_rows_per_split(256000, 3, 3200) == 512
    finally:
        ops.torch.cuda.current_device = dev
        ops._CU_COUNT.clear()
        ops._CU_COUNT.update(saved)
