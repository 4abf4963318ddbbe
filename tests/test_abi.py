"""CPU: the C-ABI library loads and exports every symbol include/*.h declares; host-side
validation and layout queries work without a GPU (no compute calls here)."""

import ctypes
import glob
import os
import re

import pytest

from conftest import REPO

from cgr_mpnn_3D._amd import native


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(REPO, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(cgr_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_loads_and_abi_version():
    lib = native.load()
    assert lib.cgr_abi_version() == native.ABI_VERSION


def test_library_was_built_from_these_sources():
    """csrc/Makefile records the SHA-256 of every source beside the library it links
    (cgr_mpnn_3D/_amd/buildinfo.py); a library stale against the tree fails here (and in
    smoke()) instead of running silently (the .so ships prebuilt)."""
    from cgr_mpnn_3D._amd import buildinfo

    if os.path.abspath(native.LIB_PATH) != os.path.abspath(
            os.path.join(os.path.dirname(buildinfo.INFO), os.path.basename(native.LIB_PATH))):
        pytest.skip("CGR_MPNN3D_LIB points at another library")
    info = buildinfo.check()
    assert info.get("sources_sha256"), "no build record beside the library: rebuild (make)"
    assert info["matches_sources"], "the library is stale against csrc/ and include/: rebuild"
    assert "gfx950" in info["flags"]


def test_every_declared_symbol_is_exported_and_bound():
    declared = _declared_functions()
    assert len(declared) >= 12
    lib = ctypes.CDLL(native.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    bound = {s[0] for s in native.SIGNATURES}
    assert declared == bound, declared ^ bound


def _cfg(F=846, Fe=14, H=400, D=4, act=0, skip=0):
    return native.CgrGnnConfig(F, Fe, H, D, act, skip)


def test_num_params_matches_state_dict_order():
    lib = native.load()
    assert lib.cgr_gnn_num_params(ctypes.byref(_cfg(D=4))) == 6 + 8
    assert lib.cgr_gnn_num_params(ctypes.byref(_cfg(D=6, skip=1))) == 6 + 12 + 6


def test_arena_and_workspace_sizes_scale():
    lib = native.load()
    c = _cfg()
    a1 = lib.cgr_gnn_arena_bytes(ctypes.byref(c), 7680, 15360, 256)
    a2 = lib.cgr_gnn_arena_bytes(ctypes.byref(c), 2 * 7680, 2 * 15360, 512)
    assert 0 < a1 < a2
    # ReLU keeps no pre-activations; SiLU does
    c_silu = _cfg(act=1)
    assert lib.cgr_gnn_arena_bytes(ctypes.byref(c_silu), 7680, 15360, 256) > a1
    w = lib.cgr_gnn_workspace_bytes(ctypes.byref(c), 7680, 15360, 256)
    assert w > 3 * 15360 * 400 * 4
    # every saved buffer is 256-byte aligned
    for name, idx in [("h", 0), ("h", 4), ("a", 4), ("hn", 0), ("perm", 0), ("status", 0)]:
        off = lib.cgr_gnn_arena_offset(ctypes.byref(c), 7680, 15360, 256, name.encode(), idx)
        assert off >= 0 and off < a1
        if name not in ("status",):
            assert off % 256 == 0
    assert lib.cgr_gnn_arena_offset(ctypes.byref(c), 7680, 15360, 256, b"pre", 1) == -1
    assert lib.cgr_gnn_arena_offset(ctypes.byref(c_silu), 7680, 15360, 256, b"pre", 1) > 0


@pytest.mark.parametrize("bad", [dict(D=0), dict(D=33), dict(H=0), dict(act=10), dict(act=-1), dict(Fe=-1)])
def test_invalid_config_is_rejected_with_message(bad):
    lib = native.load()
    c = _cfg(**bad)
    assert lib.cgr_gnn_num_params(ctypes.byref(c)) == -1
    assert lib.cgr_last_error()


def test_invalid_batch_rejected_before_any_launch():
    lib = native.load()
    c = _cfg(F=4, Fe=2, H=8, D=1)
    # odd edge count: the reference's view(E//2, 2, -1) needs pairs
    b = native.CgrBatch(1, 1, 1, None, None, 4, 3, 1)
    params = (ctypes.c_void_p * 8)(*([1] * 8))
    rc = lib.cgr_gnn_forward(ctypes.byref(c), params, ctypes.byref(b), None, 0, None, 0, 1, 1,
                             None)
    assert rc == 1 and b"even" in lib.cgr_last_error()
    b = native.CgrBatch(1, 1, 1, None, None, 4, 4, 2)  # B > 1 but no batch vector
    rc = lib.cgr_gnn_forward(ctypes.byref(c), params, ctypes.byref(b), None, 0, None, 0, 1, 1,
                             None)
    assert rc == 1


def test_fused_adam_rejects_cpu_parameters():
    import torch

    from cgr_mpnn_3D._amd.optim import FusedAdam

    p = torch.zeros(4, requires_grad=True)
    opt = FusedAdam([p], lr=1e-3, amsgrad=True)
    p.grad = torch.ones(4)
    with pytest.raises(RuntimeError, match="GPU"):
        opt.step()
    with pytest.raises(ValueError):
        FusedAdam([p], lr=-1.0)
