"""The C-ABI library: it loads, exports every entry point include/x2g.h declares, and its
host-side argument checks work without a GPU (no compute is launched here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "x2g.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(x2g_[a-z0-9_]+)\s*\(", text)))


def test_library_built_and_loads():
    from x2gnn import _lib

    assert os.path.exists(_lib.LIB_PATH), "run `make -C x2-gnn_amd` (or __graft_entry__.build())"
    lib = _lib.load()
    assert lib.x2g_abi_version() == 17


def test_every_declared_symbol_is_exported_and_bound():
    from x2gnn import _lib

    lib = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 17
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} declared in x2g.h but not bound in _lib.SIGNATURES"
    assert sorted(_lib.SIGNATURES) == syms


def test_status_strings_and_workspace_query():
    from x2gnn import _lib

    lib = _lib.load()
    assert lib.x2g_status_string(0) == b"ok"
    assert b"EINVAL" in lib.x2g_status_string(1001)
    assert b"UNSUPPORTED" in lib.x2g_status_string(1002)
    ws = lib.x2g_vertex_to_edge_workspace(20000, 2304)
    assert ws >= 4 * 2 * 20000


@pytest.mark.parametrize("name,args", [
    ("x2g_csr_rowptr", (None, -1, 4, None, None)),
    ("x2g_segment_sum", (None, None, None, -1, 128, None, None)),
    ("x2g_segment_sum", (None, None, None, 4, 0, None, None)),
    ("x2g_graph_layernorm_fwd", (None, None, -3, 128, 1e-8, None, None, None, None)),
    ("x2g_bessel_env", (None, 10, -1.0, 7, 6, None, None)),
])
def test_argument_validation_without_gpu(name, args):
    from x2gnn import _lib

    fn = getattr(_lib.load(), name)
    assert fn(*args) == 1001


@pytest.mark.parametrize("nsph,nrad", [(8, 6), (7, 17), (0, 6), (7, 0)])
def test_basis_rejects_uncompiled_shapes(nsph, nrad):
    """F_B_2D is compiled for num_spherical <= 7, num_radial <= 16 (the reference default 7 x 16)."""
    from x2gnn import _lib

    p = ctypes.c_void_p(16)  # never dereferenced: the shape check fails first
    assert _lib.load().x2g_bessel_env(p, 4, 5.0, nsph, nrad, p, None) == 1002


def test_attention_rejects_uncompiled_shapes():
    from x2gnn import _lib

    lib = _lib.load()
    p = ctypes.c_void_p(16)  # never dereferenced: the shape check fails first
    rc = lib.x2g_sbf_attention_fwd(p, p, p, p, None, None, 0, p, p, p, p, p, 4, 0, 3, 7, 42, p, p, p, p, None)
    assert rc == 1002
    rc = lib.x2g_sbf_attention_fwd(p, p, p, p, None, None, 0, p, p, p, p, p, 4, 0, 16, 8, 40, p, p, p, p, None)
    assert rc == 1002


def test_center_backward_refuses_32bit_overflow_and_host_falls_back():
    """The center backward addresses its T-row arrays with 32-bit buffer offsets: T * 512 B for S rows,
    T * heads * 8 B (the (g, a) scratch) for P rows; beyond that it returns X2G_EUNSUPPORTED before
    touching anything, and the host's predicate routes such a batch to the destination-major passes
    (which the forward then feeds with S rows) instead of failing in the backward."""
    import types

    from x2gnn import _lib, ops

    lib = _lib.load()
    p = ctypes.c_void_p(16)  # never dereferenced: the size check fails first
    big = (1 << 31) // 512  # the first T whose S rows overflow
    args = lambda sp, pp, T: (p, p, p, None, None, 0, sp, pp, p, p, p, p, p, p, p, p, p, p, 4, 16, 64, T, 16, 8,  # noqa: E731
                              p, p, p, p, None, p, None)
    assert lib.x2g_sbf_attention_bwd_center(*args(p, None, big)) == 1002
    assert lib.x2g_sbf_attention_bwd_center(*args(None, p, (1 << 31) // 128)) == 1002
    lg = types.SimpleNamespace(atom_type=object(), max_degree=16, T=big - 1)
    assert ops._center_bwd_ok(lg, 16) and ops._center_bwd_ok(lg, 16, s_rows=True)
    lg.T = big
    assert ops._center_bwd_ok(lg, 16) and not ops._center_bwd_ok(lg, 16, s_rows=True)
    lg.T = (1 << 31) // 128
    assert not ops._center_bwd_ok(lg, 16)
