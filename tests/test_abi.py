"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports every entry point
declared in include/dvcp.h, the ctypes prototypes cover them all, and the product path has no
CPU fallback (ops raise instead of computing when no GPU is present)."""
import os
import re
import subprocess

import pytest
import torch

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "dvcp.h")


def declared():
    text = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(dvcp_\w+)\s*\(", text, re.M)))


def test_header_declares_entry_points():
    names = declared()
    assert "dvcp_fps" in names and "dvcp_knn" in names and "dvcp_svd_optimization" in names
    assert len(names) >= 17


def test_library_exports_every_declared_symbol():
    import dvcp
    from dvcp import _lib
    lib = dvcp.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (dvcp_\w+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    assert sorted(_lib.exported_symbols()) == declared()
    assert lib.dvcp_abi_version() == 4


def test_ctypes_prototypes_match_header_arity():
    """Every ctypes prototype in dvcp/_lib.py has as many arguments as the header declares."""
    from dvcp import _lib
    text = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = dict(re.findall(r"(?:int|int64_t|const char\*)\s+(dvcp_\w+)\s*\(([^)]*)\)\s*;", text))
    for name, argtypes in _lib.SIGNATURES.items():
        params = protos[name].strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert n == len(argtypes), (name, n, len(argtypes))


def test_error_path_reports_message():
    import dvcp
    from dvcp import _lib
    dvcp.load_library()
    with pytest.raises(RuntimeError, match="null pointer"):
        _lib.call("dvcp_fps", 7, None, 0, 0, 0, 1, 1, 1, _lib.ctypes.c_void_p(8), _lib.ctypes.c_void_p(8), None, None)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_no_cpu_fallback():
    import dvcp
    import dvcp.pointnet2_utils as P
    x = torch.rand(1, 100, 3)
    with pytest.raises(RuntimeError, match="no GPU"):
        P.farthest_point_sample(x, 10)
    with pytest.raises(RuntimeError, match="no GPU"):
        dvcp.KNN(k=4, transpose_mode=True)(x, x)
    m = dvcp.DeepVCP(use_normal=False, fe_npoint=16).eval()
    with pytest.raises(RuntimeError):
        m(torch.rand(1, 3, 64), torch.rand(1, 3, 64), torch.eye(3, dtype=torch.float64)[None], torch.zeros(1, 3))


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU behaviour")
def test_training_guards_and_no_cpu_fallback():
    """Training mode: the whole model in training mode (batch-statistics BN in FE1), FE1.eval()
    (frozen-BN training) and a frozen FE1 all take the autograd path, which has no CPU fallback."""
    import dvcp
    m = dvcp.DeepVCP(use_normal=False, fe_npoint=16)
    args = (torch.rand(1, 3, 64), torch.rand(1, 3, 64), torch.eye(3, dtype=torch.float64)[None], torch.zeros(1, 3))
    assert m._training_mode() == (True, True)      # model.train(): batch-statistics BN
    with pytest.raises(RuntimeError, match="no GPU"):
        m(*args)
    m.FE1.eval()
    assert m._training_mode() == (True, True)      # frozen-BN training of the extractor and the head
    with pytest.raises(RuntimeError, match="no GPU"):
        m(*args)
    m.FE1.requires_grad_(False)
    assert m._training_mode() == (True, False)     # head only
    with pytest.raises(RuntimeError, match="no GPU"):
        m(*args)
    with pytest.raises(RuntimeError, match="no GPU"):
        dvcp.deepVCP_loss(torch.rand(1, 8, 3), torch.rand(1, 8, 3, requires_grad=True),
                          torch.eye(3, dtype=torch.float64)[None], torch.zeros(1, 3, 1, dtype=torch.float64), 0.5)
    with pytest.raises(RuntimeError, match="no GPU"):
        dvcp.feat_embedding_layer()(torch.rand(1, 2, 32, 35, requires_grad=True))


def test_product_never_imports_oracle():
    for dirpath, _, files in os.walk(os.path.join(PKG, "dvcp")):
        for f in files:
            if f.endswith(".py"):
                src = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f


def test_fps_pair_gating(monkeypatch):
    """The FE chain takes the paired layer-2/3 FPS launch only when asked (DVCP_FPS_PAIR=1) and
    only where it is defined: fp32, both layers picking every point, 2048..16384 points."""
    from dvcp import _lib, ops
    x = torch.zeros(2, 3, 10000)
    monkeypatch.delenv("DVCP_FPS_PAIR", raising=False)
    assert not ops.fps_pair_ok(x, 10000, 10000, pdim=2)
    monkeypatch.setenv("DVCP_FPS_PAIR", "1")
    assert ops.fps_pair_ok(x, 10000, 10000, pdim=2)
    assert not ops.fps_pair_ok(x, 9999, 10000, pdim=2)
    assert not ops.fps_pair_ok(x, 10000, 4096, pdim=2)
    assert not ops.fps_pair_ok(x.double(), 10000, 10000, pdim=2)
    assert not ops.fps_pair_ok(torch.zeros(2, 3, 1000), 1000, 1000, pdim=2)
    assert not ops.fps_pair_ok(torch.zeros(2, 3, 20000), 20000, 20000, pdim=2)
    assert _lib.load().dvcp_fps_pair_workspace_bytes(16, 10000) == 4 * (1 + 32 + 160000)


def test_fps_parts_choice_and_workspace(monkeypatch):
    """The split select's defaults (8 workgroups per cloud above 16384 fp32 points, else one unless
    DVCP_FPS_PARTS asks) and its workspace: every part's exchange slot as the kernel lays it out
    (8 header granules, one T granule per wave of a 1024-thread workgroup, 5 x 128 / S candidate
    granules, 8 bytes each), double-buffered, plus B flags and the ticket, the B x N permutation
    and the error word.  (Round 6: slots sized without the T granules overran into the flags and
    the permutation; a part starting late read another cloud's candidates as point indices.)"""
    from dvcp import _lib, ops
    monkeypatch.delenv("DVCP_FPS_PARTS", raising=False)
    assert ops.fps_parts(16384) == 1 and ops.fps_parts(10000) == 1
    assert ops.fps_parts(16385) == 8 and ops.fps_parts(65536) == 8
    assert ops.fps_parts(65537) == 1 and ops.fps_parts(40000, torch.float64) == 1
    monkeypatch.setenv("DVCP_FPS_PARTS", "4")
    assert ops.fps_parts(10000) == 4 and ops.fps_parts(1000) == 1
    for B, N in ((16, 10000), (16, 16384), (4, 65536), (3, 2048)):
        need = 0
        for S in (2, 4, 8):
            slots = B * 2 * S * (8 + 16 + 5 * (128 // S)) * 8
            flags = (B * 4 + 4 + 7) // 8 * 8
            need = max(need, slots + flags + B * N * 4 + 8)
        assert _lib.load().dvcp_fps_workspace_bytes(B, N) >= need, (B, N)


def test_graft_entry_build():
    """__graft_entry__.build(): make (nothing to do once built) and the library's ABI version
    against dvcp/_lib.py's (round 6 left a stale literal there for a while)."""
    import importlib
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if root not in sys.path:
        sys.path.insert(0, root)
    ge = importlib.import_module("__graft_entry__")
    ge.build()
