"""Kernel-level parity on the GPU: every libx2g.so operator against the reference fixtures and the
CPU oracle on the same seeded inputs (integer work bit-exact, float work within stated
tolerances)."""
import math
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden
from helpers import rel_err

from oracle import ref_cpu, triplets

pytestmark = pytest.mark.gpu


def _lg(ei_np, n, T, dev):
    from x2gnn import ops

    return ops.vertex_to_edge(torch.from_numpy(ei_np.astype(np.int64)).to(dev), n, T)


# ------------------------------------------------------------------------------ triplets
def _check_transpose(lg):
    rp, perm = (t.cpu().numpy() for t in lg.src_csr())
    src = lg.trip_src.cpu().numpy()
    assert rp[0] == 0 and rp[-1] == lg.T
    assert np.array_equal(np.sort(perm), np.arange(lg.T))            # a permutation
    assert np.all(np.diff(src[perm]) >= 0)                            # grouped by source
    np.testing.assert_array_equal(np.diff(rp), np.bincount(src, minlength=lg.E))
    for s in range(lg.E):                                             # ascending inside a group
        seg = perm[rp[s]:rp[s + 1]]
        assert np.all(np.diff(seg) > 0)


def test_vertex_to_edge_matches_reference(cuda):
    z = golden("triplets.npz")
    for case in z["cases"]:
        ei, n = z[f"{case}_edge_index"], int(z[f"{case}_num_nodes"])
        ref = z[f"{case}_trip"]
        lg = _lg(ei, n, ref.shape[1], cuda)
        np.testing.assert_array_equal(lg.trip_src.cpu().numpy(), ref[0])
        np.testing.assert_array_equal(lg.trip_dst.cpu().numpy(), ref[1])
        np.testing.assert_array_equal(lg.atom_j.cpu().numpy(), z[f"{case}_j"])
        np.testing.assert_array_equal(lg.atom_i.cpu().numpy(), z[f"{case}_i"])
        np.testing.assert_array_equal(lg.atom_k.cpu().numpy(), z[f"{case}_k"])
        rp = lg.trip_rowptr.cpu().numpy()
        np.testing.assert_array_equal(np.diff(rp), np.bincount(ref[1], minlength=ei.shape[1]))
        np.testing.assert_array_equal(lg.atom_rowptr.cpu().numpy(),
                                      np.searchsorted(ei[0], np.arange(n + 1), side="left"))
        if case in ("s160", "directed"):
            _check_transpose(lg)


def test_vertex_to_edge_full_batch_vs_oracle(cuda):
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(128, "S160", seed=3))
    ei = b.edge_index.numpy()
    T = int(b._meta["triplets"].sum())
    lg = _lg(ei, b.num_nodes, T, cuda)
    trip, j, i, k = triplets.vertex_to_edge(ei, b.num_nodes)
    np.testing.assert_array_equal(lg.trip_src.cpu().numpy(), trip[0])
    np.testing.assert_array_equal(lg.trip_dst.cpu().numpy(), trip[1])
    np.testing.assert_array_equal(lg.atom_k.cpu().numpy(), k)
    rp, perm = (t.cpu().numpy() for t in lg.src_csr())
    assert np.all(np.diff(trip[0][perm]) >= 0) and np.array_equal(np.sort(perm), np.arange(T))


def test_vertex_to_edge_edge_cases(cuda):
    from x2gnn import ops

    # no edges at all
    lg = ops.vertex_to_edge(torch.zeros(2, 0, dtype=torch.int64, device=cuda), 5, 0)
    assert lg.T == 0 and lg.trip_rowptr.cpu().tolist() == [0]
    assert lg.atom_rowptr.cpu().tolist() == [0] * 6
    # one bond (a <-> b): no triplets; isolated trailing atoms
    ei = np.array([[0, 1], [1, 0]])
    lg = _lg(ei, 4, 0, cuda)
    assert lg.trip_rowptr.cpu().tolist() == [0, 0, 0]
    assert lg.atom_rowptr.cpu().tolist() == [0, 1, 2, 2, 2]
    # a star with a hub of degree 70 (> one 64-lane chunk)
    hub = np.array([[0] * 70 + list(range(1, 71)), list(range(1, 71)) + [0] * 70])
    order = np.lexsort((hub[1], hub[0]))
    hub = hub[:, order]
    trip, *_ = triplets.vertex_to_edge(hub, 71)
    lg = _lg(hub, 71, trip.shape[1], cuda)
    np.testing.assert_array_equal(lg.trip_src.cpu().numpy(), trip[0])
    _check_transpose(lg)


def _sym_vs_generic(ei, n, T, cuda):
    """x2g_vertex_to_edge_sym / x2g_line_graph_transpose_sym and x2g_line_graph_sym_build against the
    generic builder and transpose on the same symmetric graph: every output bit-for-bit."""
    from x2gnn import ops

    e = torch.from_numpy(ei.astype(np.int64)).to(cuda)
    gen = ops.vertex_to_edge(e, n, T)
    ei32 = ops._i32(e)
    # the two entry points in turn (transpose built on first use) and x2g_line_graph_sym_build (both at once)
    for wt in (False, True):
        sym = ops.LineGraph(ei32[0].contiguous(), ei32[1].contiguous(), n, T, symmetric=True, with_transpose=wt)
        assert (sym._src_rowptr is not None) == wt
        for name in ("atom_rowptr", "trip_rowptr", "trip_src", "trip_dst", "atom_j", "atom_i", "atom_k"):
            assert torch.equal(getattr(gen, name), getattr(sym, name)), (name, wt)
        for a, b in zip(gen.src_csr(), sym.src_csr()):
            assert torch.equal(a, b), wt
        assert torch.equal(gen.src_dst, sym.src_dst), wt
    # src_dst = trip_dst[src_perm]; and the source-uniform edge row the fold pass relies on: every
    # triplet of source s = (b->k) goes into a destination (a->b) whose destination atom is s's source
    perm = sym.src_csr()[1].long()
    assert torch.equal(sym.src_dst, sym.trip_dst[perm])
    if sym.T:
        rp = sym.src_csr()[0].long()
        src_of_pos = torch.repeat_interleave(torch.arange(sym.E, device=cuda), rp[1:] - rp[:-1])
        assert torch.equal(sym.edge_dst.long()[sym.src_dst.long()], sym.edge_src.long()[src_of_pos])
    # the center-atom outputs: edge_rev[e] is the reverse edge, rev_trip[s] the triplet block start of
    # s's reverse (trip_rowptr[edge_rev[s]])
    if sym.E:
        rev = sym.edge_rev.long()
        assert torch.equal(sym.edge_src.long()[rev], sym.edge_dst.long())
        assert torch.equal(sym.edge_dst.long()[rev], sym.edge_src.long())
        assert torch.equal(rev[rev], torch.arange(sym.E, device=cuda))
        assert torch.equal(sym.rev_trip, sym.trip_rowptr[rev])
    return sym


def test_symmetric_builder_and_transpose_equal_generic(cuda):
    """The degree-count builder and the direct (no atomics, no sort) transpose for symmetric edge
    sets: the symmetric fixtures, a full config-2 batch (collate marks it symmetric), a hub of
    degree 70, isolated atoms, no edges, and a graph larger than the one-workgroup scan
    (E > 32768: the multi-workgroup scan path)."""
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    z = golden("triplets.npz")
    for case in z["cases"]:
        ei, n = z[f"{case}_edge_index"], int(z[f"{case}_num_nodes"])
        fwd = set(zip(ei[0].tolist(), ei[1].tolist()))
        if all((b, a) in fwd for a, b in fwd):
            _sym_vs_generic(ei, n, z[f"{case}_trip"].shape[1], cuda)
    b = collate(synthetic_molecules(128, "S160", seed=3))
    assert b._store["_x2g_symmetric"]
    _sym_vs_generic(b.edge_index.numpy(), b.num_nodes, int(b._meta["triplets"].sum()), cuda)
    hub = np.array([[0] * 70 + list(range(1, 71)), list(range(1, 71)) + [0] * 70])
    hub = hub[:, np.lexsort((hub[1], hub[0]))]
    _sym_vs_generic(hub, 75, triplets.vertex_to_edge(hub, 75)[0].shape[1], cuda)
    _sym_vs_generic(np.zeros((2, 0), dtype=np.int64), 3, 0, cuda)
    big = collate(synthetic_molecules(1800, "S160", seed=5))
    assert big.edge_index.shape[1] > 32768
    _sym_vs_generic(big.edge_index.numpy(), big.num_nodes, int(big._meta["triplets"].sum()), cuda)


def test_per_molecule_builder_equals_whole_batch(cuda):
    """x2g_vertex_to_edge_sym_mol (row pointers one workgroup per molecule, from the molecules' atom / edge
    pointers and triplet counts) == x2g_vertex_to_edge_sym over the whole batch, every output bit for bit,
    and the transpose it leaves to src_csr too: a config-2 batch, one larger than the one-workgroup scan,
    and a batch with one-atom and two-atom molecules (no triplets) between ordinary ones, first and last."""
    from x2gnn import ops
    from x2gnn.data import collate
    from x2gnn.synth import molecule_from_geometry, synthetic_molecules

    rng = np.random.default_rng(0)
    lone = molecule_from_geometry(np.array([6]), np.zeros((1, 3)), feat_rng=rng, y=0.0)
    pair = molecule_from_geometry(np.array([1, 1]), np.array([[0.0, 0, 0], [0.74, 0, 0]]), feat_rng=rng, y=0.0)
    cases = [synthetic_molecules(128, "S160", seed=21), synthetic_molecules(1800, "S160", seed=22),
             [lone, pair] + synthetic_molecules(5, "S160", seed=23) + [pair, lone]]
    for mols in cases:
        b = collate(mols).to(cuda)
        st = b._store
        n, T = b.num_nodes, int(b._meta["triplets"].sum())
        ref = ops.LineGraph(st["_x2g_edge_src"], st["_x2g_edge_dst"], n, T, symmetric=True, with_transpose=False)
        mol = ops.LineGraph(st["_x2g_edge_src"], st["_x2g_edge_dst"], n, T, symmetric=True,
                            molecules=(st["_x2g_mol_ptr"], st["_x2g_line_ptr"], st["_x2g_mol_trips"],
                                       st["_x2g_max_mol_atoms"]))
        assert mol._src_rowptr is None  # (the center-atom backward never reads the transpose)
        for name in ("atom_rowptr", "trip_rowptr", "trip_src", "trip_dst", "atom_j", "atom_i", "atom_k", "edge_rev",
                     "rev_trip"):
            assert torch.equal(getattr(ref, name), getattr(mol, name)), name
        for x, y in zip(ref.src_csr(), mol.src_csr()):
            assert torch.equal(x, y)


def test_csr_rowptr(cuda):
    from x2gnn import ops

    keys = np.array([0, 0, 2, 2, 2, 5, 7, 7])
    rp = ops.csr_rowptr(torch.from_numpy(keys).to(cuda), 9).cpu().numpy()
    np.testing.assert_array_equal(rp, np.searchsorted(keys, np.arange(10), side="left"))


# ------------------------------------------------------------------------------ basis
BASIS_TOL = [1e-5, 1e-5, 1e-5, 1e-4, 1e-3, 5e-3, 3e-2]  # per l: the reference's fp32 cancellation


def test_spherical_basis_vs_reference(cuda):
    from x2gnn import ops

    z = golden("basis.npz")
    ei = z["edge_index"].astype(np.int64)
    n = int(z["nodes"].sum())
    lg = _lg(ei, n, z["trip"].shape[1], cuda)
    d = torch.from_numpy(z["dist"]).to(cuda)
    rbf_env = ops.bessel_env(d)
    pos = torch.from_numpy(z["atom_pos"]).to(cuda)
    sbf, cos_t = ops.spherical_basis(pos, lg, rbf_env, want_cos=True)
    sbf = sbf.cpu().numpy()
    for l in range(7):
        blk = slice(6 * l, 6 * l + 6)
        assert np.abs(sbf[:, blk] - z["sbf"][:, blk]).max() < BASIS_TOL[l], l
    np.testing.assert_allclose(cos_t.cpu().numpy(), np.cos(z["theta"]), atol=2e-6)
    # the theta-input entry point (F_B_2D.forward(d, Angles, edge_index_1) signature)
    sbf2 = ops.spherical_basis_from_angles(torch.from_numpy(z["theta"]).to(cuda), lg.trip_src, rbf_env).cpu().numpy()
    for l in range(7):
        blk = slice(6 * l, 6 * l + 6)
        assert np.abs(sbf2[:, blk] - z["sbf"][:, blk]).max() < BASIS_TOL[l], l
    # against the fp64 oracle, l <= 3 the reference formula is accurate to ~1e-6
    orc = ref_cpu.spherical_basis(torch.from_numpy(z["dist"]), torch.from_numpy(z["theta"]),
                                  torch.from_numpy(z["trip"][0].astype(np.int64))).numpy()
    assert np.abs(sbf[:, :24] - orc[:, :24]).max() < 1e-4


def test_spherical_basis_7x16_vs_reference(cuda):
    """F_B_2D(7, 16) (the reference's default xgnn_poly basis): x2g_edge_basis / x2g_bessel_env /
    x2g_spherical_basis at num_radial 16 against the reference's own output (basis_7x16.npz), and
    RadialBasis(16) times the envelope."""
    from x2gnn import ops

    z = golden("basis_7x16.npz")
    ei = z["edge_index"].astype(np.int64)
    n = int(z["nodes"].sum())
    lg = _lg(ei, n, z["trip"].shape[1], cuda)
    pos = torch.from_numpy(z["atom_pos"]).to(cuda)
    freq = (math.pi * torch.arange(1, 17, dtype=torch.float32)).to(cuda)
    dist, env, rbf, bes = ops.edge_basis(pos, lg, freq, 5.0, 7, 16)
    np.testing.assert_allclose(dist.cpu().numpy(), z["dist"], rtol=2e-6, atol=2e-6)
    np.testing.assert_allclose(rbf.cpu().numpy(), z["rbf"], rtol=1e-5, atol=5e-5)
    for radial in (bes, ops.bessel_env(dist, 5.0, 7, 16)):
        sbf = ops.spherical_basis(pos, lg, radial, num_spherical=7, num_radial=16).cpu().numpy()
        assert sbf.shape == z["sbf"].shape == (lg.T, 112)
        for l in range(7):
            blk = slice(16 * l, 16 * l + 16)
            # the 16-wide blocks reach |sbf| ~ 15 (vs ~ 3 at 7 x 6): a relative term of 2 ulp-ish on top
            tol = BASIS_TOL[l] + 2e-6 * np.abs(z["sbf"][:, blk]).max()
            assert np.abs(sbf[:, blk] - z["sbf"][:, blk]).max() < tol, l
    sbf2 = ops.spherical_basis_from_angles(torch.from_numpy(z["theta"]).to(cuda), lg.trip_src, bes, 7, 16).cpu().numpy()
    for l in range(7):
        blk = slice(16 * l, 16 * l + 16)
        tol = BASIS_TOL[l] + 2e-6 * np.abs(z["sbf"][:, blk]).max()
        assert np.abs(sbf2[:, blk] - z["sbf"][:, blk]).max() < tol, l


def test_radial_parts_vs_reference(cuda):
    from x2gnn.layers import RadialBasis, poly_envelop

    z = golden("basis.npz")
    d = torch.from_numpy(z["dist"]).to(cuda)
    env = poly_envelop(5.0, 5)(d)
    # near d = cutoff the envelope is a difference of O(50) terms: absolute slack of a few ulps of them
    np.testing.assert_allclose(env.cpu().numpy(), z["env"], rtol=2e-6, atol=2e-5)
    rbf = RadialBasis(6, 5.0).to(cuda)(d) * env[:, None]
    np.testing.assert_allclose(rbf.detach().cpu().numpy(), z["rbf"], rtol=1e-5, atol=2e-5)


# ------------------------------------------------------------------------------ segments
def _rowptr_with_empties(rng, n_seg, max_len):
    lens = rng.integers(0, max_len + 1, size=n_seg)
    lens[rng.random(n_seg) < 0.2] = 0
    return np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)


@pytest.mark.parametrize("D", [1, 6, 32, 128, 256])
@pytest.mark.parametrize("with_mul", [False, True])
def test_segment_sum_and_adjoint(cuda, D, with_mul):
    from x2gnn import ops

    rng = np.random.default_rng(D)
    rp = _rowptr_with_empties(rng, 333, 40)
    R = int(rp[-1])
    x = torch.randn(R, D, dtype=torch.float64)
    m = torch.randn(R, D, dtype=torch.float64) if with_mul else None
    seg = np.repeat(np.arange(333), np.diff(rp))
    ref = torch.zeros(333, D, dtype=torch.float64).index_add_(0, torch.from_numpy(seg), x * m if with_mul else x)
    xg = x.float().to(cuda).requires_grad_(True)
    mg = m.float().to(cuda).requires_grad_(True) if with_mul else None
    out = ops.segment_sum(xg, torch.from_numpy(rp).to(cuda), 333, mul=mg)
    assert rel_err(out.detach().cpu().numpy(), ref.numpy()) < 1e-5
    g = torch.randn(333, D)
    out.backward(g.to(cuda))
    gx = g.double()[torch.from_numpy(seg)]
    np.testing.assert_allclose(xg.grad.cpu().numpy(), (gx * m if with_mul else gx).numpy(), rtol=1e-5, atol=1e-5)
    if with_mul:
        np.testing.assert_allclose(mg.grad.cpu().numpy(), (gx * x).numpy(), rtol=1e-5, atol=1e-5)


def test_segment_sum_is_deterministic(cuda):
    from x2gnn import ops

    rng = np.random.default_rng(0)
    rp = torch.from_numpy(_rowptr_with_empties(rng, 5000, 30)).to(cuda)
    x = torch.randn(int(rp[-1]), 128, device=cuda)
    a = ops.segment_sum(x, rp, 5000)
    b = ops.segment_sum(x, rp, 5000)
    assert torch.equal(a, b)


def test_segment_softmax_vs_oracle(cuda):
    from x2gnn import ops

    rng = np.random.default_rng(1)
    rp = _rowptr_with_empties(rng, 200, 25)
    R = int(rp[-1])
    seg = torch.from_numpy(np.repeat(np.arange(200), np.diff(rp)))
    src = (3 * torch.randn(R, 16)).requires_grad_(True)
    ref = ref_cpu.pyg_softmax(src, seg, 200)
    g = torch.randn(R, 16)
    ref.backward(g)
    sg = src.detach().to(cuda).requires_grad_(True)
    out = ops.segment_softmax(sg, torch.from_numpy(rp).to(cuda), 200)
    out.backward(g.to(cuda))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(sg.grad.cpu().numpy(), src.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_graph_layernorm_vs_oracle(cuda):
    from x2gnn import ops

    counts = np.array([162, 0, 1, 288, 40, 2037])  # includes an empty and a one-row molecule
    rp = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    batch = torch.from_numpy(np.repeat(np.arange(len(counts)), counts))
    x = (torch.randn(int(rp[-1]), 128) * 3 + 1).requires_grad_(True)
    ref = ref_cpu.graph_layer_norm(x, batch, 1e-8)
    g = torch.randn_like(ref)
    ref.backward(g)
    xg = x.detach().to(cuda).requires_grad_(True)
    out = ops.graph_layer_norm(xg, torch.from_numpy(rp).to(cuda), len(counts), 1e-8)
    out.backward(g.to(cuda))
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(xg.grad.cpu().numpy(), x.grad.numpy(), rtol=1e-3, atol=1e-5)


def test_graph_layernorm_bwd_split_equals_one_block(cuda):
    """x2g_graph_layernorm_bwd_ex (4 workgroups per segment: stats pass + apply pass) against the
    one-workgroup-per-segment x2g_graph_layernorm_bwd on ragged segments (empty, one row, QM9- and
    AID-sized, one past the register-resident capacity); bitwise run to run."""
    from x2gnn._lib import call, load, ptr, stream_ptr

    counts = np.array([165, 0, 1, 3, 288, 2037, 257, 7])
    rp = torch.from_numpy(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)).to(cuda)
    R, G = int(counts.sum()), len(counts)
    g = torch.Generator(device=cuda).manual_seed(5)
    y = torch.randn(R, 128, device=cuda, generator=g)
    dy = torch.randn(R, 128, device=cuda, generator=g)
    rstd = torch.rand(G, device=cuda, generator=g) + 0.5
    ref = torch.empty_like(y)
    call("x2g_graph_layernorm_bwd", ptr(y), ptr(dy), ptr(rstd), ptr(rp), G, 128, ptr(ref), stream_ptr())
    wsb = int(load().x2g_graph_layernorm_bwd_workspace(G))
    ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
    outs = []
    for _ in range(2):
        dx = torch.full_like(y, float("nan"))
        call("x2g_graph_layernorm_bwd_ex", ptr(y), ptr(dy), ptr(rstd), ptr(rp), G, 128, ptr(dx), ptr(ws), wsb,
             stream_ptr())
        outs.append(dx)
    torch.testing.assert_close(outs[0], ref, rtol=1e-5, atol=1e-5)
    assert torch.equal(outs[0], outs[1])


# ------------------------------------------------------------------------------ attention
def _product_conv(z, cuda):
    from weights import load_seeded
    from x2gnn import SBFTransformerConv

    conv = SBFTransformerConv(in_channels=128, out_channels=8, heads=16, sbf_dim=42, rbf_dim=6, dropout=0,
                              edge_dim=128)
    load_seeded(conv, int(z["weight_seed"]))
    return conv.to(cuda)


def test_conv_layer_vs_reference(cuda):
    """Drop-in SBFTransformerConv.forward(sbf, rbf, x, edge_index, edge_attr), per-triplet edge_attr."""
    z = golden("conv1.npz")
    conv = _product_conv(z, cuda)
    x = torch.from_numpy(z["conv_x"]).to(cuda).requires_grad_(True)
    ea = torch.from_numpy(z["conv_edge_attr"]).to(cuda).requires_grad_(True)
    out = conv(torch.from_numpy(z["sbf"]).to(cuda), torch.from_numpy(z["rbf"]).to(cuda), x,
               torch.from_numpy(z["trip"].astype(np.int64)).to(cuda), ea)
    assert rel_err(out.detach().cpu().numpy(), z["out"]) < 1e-5
    (out * torch.from_numpy(z["upstream"]).to(cuda)).sum().backward()
    assert rel_err(x.grad.cpu().numpy(), z["grad_x"]) < 1e-4
    assert rel_err(ea.grad.cpu().numpy(), z["grad_edge_attr"]) < 1e-4
    for n, p in conv.named_parameters():
        if n == "lin_key.bias":  # analytically zero: compare on the scale of the weight gradient
            assert np.abs(p.grad.cpu().numpy()).max() < 1e-5 * np.abs(z["grad.lin_key.weight"]).max()
            continue
        assert rel_err(p.grad.cpu().numpy(), z["grad." + n]) < 1e-4, n


def test_conv_attention_weights(cuda):
    z = golden("conv1.npz")
    conv = _product_conv(z, cuda)
    trip = torch.from_numpy(z["trip"].astype(np.int64)).to(cuda)
    out, (ei, alpha) = conv(torch.from_numpy(z["sbf"]).to(cuda), torch.from_numpy(z["rbf"]).to(cuda),
                            torch.from_numpy(z["conv_x"]).to(cuda), trip,
                            torch.from_numpy(z["conv_edge_attr"]).to(cuda), return_attention_weights=True)
    a = alpha.cpu().numpy()
    sums = np.zeros((z["conv_x"].shape[0], 16))
    np.add.at(sums, z["trip"][1], a)
    has = np.bincount(z["trip"][1], minlength=sums.shape[0]) > 0
    np.testing.assert_allclose(sums[has], 1.0, atol=1e-5)


def test_conv_accepts_unsorted_triplets(cuda):
    """PyG's propagate takes triplets in any order: the drop-in conv on a shuffled edge_index (sbf
    and per-triplet edge_attr rows shuffled alike) equals the reference's sorted-order output and
    gradients (the same per-destination sums up to summation order), and its attention weights come
    back in the caller's order."""
    z = golden("conv1.npz")
    conv = _product_conv(z, cuda)
    T = z["trip"].shape[1]
    perm = torch.from_numpy(np.random.default_rng(4).permutation(T)).to(cuda)
    trip = torch.from_numpy(z["trip"].astype(np.int64)).to(cuda)
    sbf = torch.from_numpy(z["sbf"]).to(cuda)
    rbf = torch.from_numpy(z["rbf"]).to(cuda)
    x = torch.from_numpy(z["conv_x"]).to(cuda).requires_grad_(True)
    ea = torch.from_numpy(z["conv_edge_attr"]).to(cuda)
    ea_p = ea.index_select(0, perm).requires_grad_(True)
    out, (ei, alpha) = conv(sbf.index_select(0, perm), rbf, x, trip.index_select(1, perm), ea_p,
                            return_attention_weights=True)
    assert rel_err(out.detach().cpu().numpy(), z["out"]) < 1e-5
    assert torch.equal(ei, trip.index_select(1, perm))
    _, (_, alpha_sorted) = conv(sbf, rbf, x.detach(), trip, ea, return_attention_weights=True)
    torch.testing.assert_close(alpha, alpha_sorted.index_select(0, perm), rtol=1e-6, atol=1e-7)
    (out * torch.from_numpy(z["upstream"]).to(cuda)).sum().backward()
    assert rel_err(x.grad.cpu().numpy(), z["grad_x"]) < 1e-4
    inv = torch.argsort(perm)
    assert rel_err(ea_p.grad.index_select(0, inv).cpu().numpy(), z["grad_edge_attr"]) < 1e-4


def test_scatter_add_any_index_order(cuda):
    """ops.scatter_add == torch_scatter.scatter_add(src, index, dim=0, dim_size) for a shuffled
    index with empty segments (fp64 torch reference), forward and the gradient of src."""
    from x2gnn import ops

    g = torch.Generator().manual_seed(8)
    idx = torch.randint(0, 50, (900,), generator=g)
    idx[idx == 7] = 8  # an empty segment
    src = torch.randn(900, 64, generator=g)
    ref = torch.zeros(60, 64, dtype=torch.float64).index_add_(0, idx, src.double())
    s = src.to(cuda).requires_grad_(True)
    out = ops.scatter_add(s, idx.to(cuda), 60)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-5, atol=1e-5)
    up = torch.randn(60, 64, generator=g)
    (out * up.to(cuda)).sum().backward()
    torch.testing.assert_close(s.grad.cpu(), up.index_select(0, idx), rtol=0, atol=0)


def test_index_plan_reused_across_scatter_and_softmax(cuda):
    """One prebuilt IndexPlan serves scatter_add, scatter_mean and softmax (as MessagePassing reuses
    edge_index[1]) with the same results as the raw-index calls; a plan built for another row count is
    refused before any kernel reads through its permutation."""
    from x2gnn import ops

    g = torch.Generator().manual_seed(21)
    idx = torch.randint(0, 30, (500,), generator=g)
    idx[idx == 11] = 12  # an empty segment
    src = torch.randn(500, 16, generator=g).to(cuda)
    ic = idx.to(cuda)
    plan = ops.IndexPlan(ic, 32)
    assert torch.equal(ops.scatter_add(src, plan, 32), ops.scatter_add(src, ic, 32))
    assert torch.equal(ops.scatter_mean(src, plan), ops.scatter_mean(src, ic, 32))
    assert torch.equal(ops.softmax(src, plan), ops.softmax(src, ic, num_nodes=32))
    s = src.clone().requires_grad_(True)
    ops.scatter_add(s, plan, 32).sum().backward()
    assert float(s.grad.sub(1.0).abs().max()) == 0.0
    with pytest.raises(ValueError):
        ops.scatter_add(src[:499], plan, 32)
    with pytest.raises(ValueError):
        ops.softmax(src[:499], plan)
    with pytest.raises(ValueError):
        ops.scatter_add(src, plan, 31)


@pytest.mark.parametrize("D", [1, 3, 16, 128, 256])
@pytest.mark.parametrize("order", ["shuffled", "sorted"])
def test_scatter_mean_any_index_order(cuda, D, order):
    """ops.scatter_mean == torch_scatter.scatter_mean(src, index, dim=0, dim_size) (readout.py:69):
    sum / max(count, 1), empty segments 0; any index order; the gradient of src is g[index] / count.
    (fp64 torch restatement of scatter_mean as the reference, torch_scatter itself not being here.)"""
    from x2gnn import ops

    g = torch.Generator().manual_seed(9 + D)
    idx = torch.randint(0, 40, (700,), generator=g)
    idx[idx == 5] = 6  # an empty segment
    if order == "sorted":
        idx = idx.sort().values
    src = torch.randn(700, D, generator=g) if D > 1 else torch.randn(700, generator=g)
    s2 = src.double().reshape(700, -1)
    cnt = torch.zeros(45, dtype=torch.float64).index_add_(0, idx, torch.ones(700, dtype=torch.float64))
    ref = torch.zeros(45, s2.shape[1], dtype=torch.float64).index_add_(0, idx, s2) / cnt.clamp(min=1)[:, None]
    s = src.to(cuda).requires_grad_(True)
    out = ops.scatter_mean(s, idx.to(cuda), 45)
    assert out.shape == ((45, D) if D > 1 else (45,))
    torch.testing.assert_close(out.double().cpu().reshape(45, -1), ref, rtol=1e-5, atol=1e-6)
    assert float(out.detach().reshape(45, -1)[5].abs().max()) == 0.0
    up = torch.randn(out.shape, generator=g)
    (out * up.to(cuda)).sum().backward()
    want = (up.double().reshape(45, -1) / cnt.clamp(min=1)[:, None]).index_select(0, idx)
    torch.testing.assert_close(s.grad.double().cpu().reshape(700, -1), want, rtol=1e-6, atol=1e-7)


def test_softmax_index_form_vs_oracle(cuda):
    """ops.softmax(src, index, num_nodes) == PyG utils.softmax (sbftransformer_conv.py:151; the
    oracle's restatement, max shift and + 1e-16) for a shuffled index with empty groups, [R] and
    [R, H], forward and backward; and equal to the sorted-index (CSR) form row for row."""
    from x2gnn import ops

    g = torch.Generator().manual_seed(12)
    idx = torch.randint(0, 60, (1500,), generator=g)
    idx[idx == 3] = 4
    for shape in ((1500, 16), (1500,)):
        src = (3 * torch.randn(*shape, generator=g)).requires_grad_(True)
        ref = ref_cpu.pyg_softmax(src, idx, 64)
        up = torch.randn(*shape, generator=g)
        ref.backward(up)
        sg = src.detach().to(cuda).requires_grad_(True)
        out = ops.softmax(sg, idx.to(cuda), num_nodes=64)
        out.backward(up.to(cuda))
        np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(sg.grad.cpu().numpy(), src.grad.numpy(), rtol=1e-4, atol=1e-6)
    order = torch.argsort(idx, stable=True)
    srt = idx[order]
    rp = torch.from_numpy(np.searchsorted(srt.numpy(), np.arange(65)).astype(np.int32)).to(cuda)
    x = torch.randn(1500, 16, device=cuda)
    a = ops.softmax(x, idx.to(cuda), num_nodes=64)
    b = ops.softmax(x[order.to(cuda)], ptr=rp)
    assert torch.equal(a[order.to(cuda)], b)


def test_scatter_ops_are_capture_safe(cuda):
    """The index-form drop-ins read nothing back from the device: scatter_add / scatter_mean /
    softmax with a fresh unsorted index record into a HIP graph and replay to the eager values."""
    from x2gnn import ops

    g = torch.Generator(device=cuda).manual_seed(3)
    idx = torch.randint(0, 30, (500,), device=cuda, generator=g)
    src = torch.randn(500, 32, device=cuda, generator=g)
    eager = (ops.scatter_add(src, idx, 30), ops.scatter_mean(src, idx, 30), ops.softmax(src, idx, num_nodes=30))
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        ops.scatter_add(src, idx, 30)  # (warm-up on a side stream, as torch.cuda.graph asks)
    torch.cuda.current_stream().wait_stream(side)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        outs = (ops.scatter_add(src, idx, 30), ops.scatter_mean(src, idx, 30), ops.softmax(src, idx, num_nodes=30))
    graph.replay()
    torch.cuda.synchronize()
    for a, b in zip(outs, eager):
        assert torch.equal(a, b)


def test_conv_assume_sorted_flags_violation_without_sync(cuda):
    """assume_sorted=True skips the device sort: on the reference's (sorted) order the output equals
    the default path's; on a shuffled order the violation is flagged on the line graph's device
    status (read here, after the fact) and nothing faults."""
    from x2gnn import ops

    z = golden("conv1.npz")
    conv = _product_conv(z, cuda)
    trip = torch.from_numpy(z["trip"].astype(np.int64)).to(cuda)
    sbf, rbf = torch.from_numpy(z["sbf"]).to(cuda), torch.from_numpy(z["rbf"]).to(cuda)
    x, ea = torch.from_numpy(z["conv_x"]).to(cuda), torch.from_numpy(z["conv_edge_attr"]).to(cuda)
    with torch.no_grad():
        a = conv(sbf, rbf, x, trip, ea)
        b = conv(sbf, rbf, x, trip, ea, assume_sorted=True)
    torch.testing.assert_close(a, b, rtol=0, atol=0)
    lg = ops.LineGraph.from_triplets(trip, x.shape[0])
    assert not lg.order_violated()
    perm = torch.from_numpy(np.random.default_rng(2).permutation(trip.shape[1])).to(cuda)
    bad = ops.LineGraph.from_triplets(trip.index_select(1, perm), x.shape[0])
    rp = bad.trip_rowptr.cpu().numpy()
    assert bad.order_violated() and rp.min() >= 0 and rp.max() <= trip.shape[1]
    with torch.no_grad():
        out = conv(sbf.index_select(0, perm), rbf, x, trip.index_select(1, perm), ea.index_select(0, perm),
                   line_graph=bad)
    torch.cuda.synchronize()
    assert out.shape == a.shape


def test_checked_rowptr_matches_plain(cuda):
    """x2g_csr_rowptr_checked == x2g_csr_rowptr on sorted keys (empty segments, keys ending early),
    status 0; an out-of-range key sets the status."""
    from x2gnn import ops

    keys = torch.tensor([0, 0, 2, 2, 2, 5, 7, 7], dtype=torch.int32, device=cuda)
    rp, st = ops.csr_rowptr_checked(keys, 10)
    assert torch.equal(rp, ops.csr_rowptr(keys, 10)) and int(st) == 0
    _, st = ops.csr_rowptr_checked(torch.tensor([0, 1, 12], dtype=torch.int32, device=cuda), 10)
    assert int(st) == 1
    rp, st = ops.csr_rowptr_checked(torch.empty(0, dtype=torch.int32, device=cuda), 4)
    assert rp.tolist() == [0, 0, 0, 0, 0] and int(st) == 0


def test_per_destination_edge_table_equals_per_triplet(cuda):
    """EDGE_PER_DST (table row per destination) == EDGE_PER_TRIPLET with the expanded rows."""
    from x2gnn import ops

    z = golden("conv1.npz")
    conv = _product_conv(z, cuda)
    trip = torch.from_numpy(z["trip"].astype(np.int64)).to(cuda)
    E = z["conv_x"].shape[0]
    g = torch.Generator().manual_seed(3)
    table = torch.randn(10, 128, generator=g).to(cuda)
    row = torch.randint(1, 10, (E,), generator=g).to(cuda)
    sbf = torch.from_numpy(z["sbf"]).to(cuda)
    rbf = torch.from_numpy(z["rbf"]).to(cuda)
    x = torch.from_numpy(z["conv_x"]).to(cuda)
    t1 = table.clone().requires_grad_(True)
    a = conv(sbf, rbf, x, trip, t1.index_select(0, row.index_select(0, trip[1])))
    t2 = table.clone().requires_grad_(True)
    lg = ops.LineGraph.from_triplets(trip, E)
    b = conv(sbf, rbf, x, trip, t2, line_graph=lg, edge_row=row)
    assert rel_err(b.detach().cpu().numpy(), a.detach().cpu().numpy()) < 1e-5
    up = torch.randn(E, 128, generator=g).to(cuda)
    (a * up).sum().backward()
    (b * up).sum().backward()
    assert rel_err(t2.grad.cpu().numpy(), t1.grad.cpu().numpy()) < 1e-4


def test_conv_small_width_vs_oracle(cuda):
    """D=32, H=4 (the reduced-width configuration of model_small) against the oracle conv."""
    from weights import load_seeded
    from x2gnn import SBFTransformerConv

    z = golden("conv1.npz")
    E, T = z["conv_x"].shape[0], z["trip"].shape[1]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(E, 32, generator=g)
    ea = torch.randn(T, 32, generator=g)
    sbf, rbf = torch.from_numpy(z["sbf"]), torch.from_numpy(z["rbf"])
    trip = torch.from_numpy(z["trip"].astype(np.int64))
    orc = ref_cpu.SBFTransformerConv(32, 4, 42, 6, 32)
    load_seeded(orc, 5)
    xr, er = x.clone().requires_grad_(True), ea.clone().requires_grad_(True)
    ref = orc(sbf, rbf, xr, trip, er)
    up = torch.randn(E, 32, generator=g)
    (ref * up).sum().backward()
    conv = SBFTransformerConv(32, 8, heads=4, sbf_dim=42, rbf_dim=6, edge_dim=32)
    load_seeded(conv, 5)
    conv = conv.to(cuda)
    xg, eg = x.to(cuda).requires_grad_(True), ea.to(cuda).requires_grad_(True)
    out = conv(sbf.to(cuda), rbf.to(cuda), xg, trip.to(cuda), eg)
    (out * up.to(cuda)).sum().backward()
    assert rel_err(out.detach().cpu().numpy(), ref.detach().numpy()) < 1e-5
    assert rel_err(xg.grad.cpu().numpy(), xr.grad.numpy()) < 1e-4
    assert rel_err(eg.grad.cpu().numpy(), er.grad.numpy()) < 1e-4
    assert rel_err(conv.lin_sbf.weight.grad.cpu().numpy(), orc.lin_sbf.weight.grad.numpy()) < 1e-4


# ------------------------------------------------------------------------------ dense layers
@pytest.mark.parametrize("R,O,I", [(21058, 128, 128), (194060, 128, 42), (1000, 256, 338), (77, 1, 128),
                                   (5, 128, 6), (130, 128, 10), (0, 128, 128), (1001, 42, 128), (333, 6, 7)])
def test_linear_wgrad_vs_fp64(cuda, R, O, I):
    from x2gnn import ops

    g = torch.Generator().manual_seed(R + O + I)
    dy = torch.randn(R, O, generator=g, dtype=torch.float64)
    x = torch.randn(R, I, generator=g, dtype=torch.float64)
    dw, db = ops.linear_wgrad(dy.float().to(cuda), x.float().to(cuda))
    ref_w, ref_b = dy.t() @ x, dy.sum(0)
    scale = max(1.0, float(np.sqrt(max(R, 1))))  # random-sign sums grow like sqrt(R)
    np.testing.assert_allclose(dw.cpu().numpy(), ref_w.numpy(), atol=2e-5 * scale, rtol=1e-5)
    np.testing.assert_allclose(db.cpu().numpy(), ref_b.numpy(), atol=2e-5 * scale, rtol=1e-5)
    dw2, _ = ops.linear_wgrad(dy.float().to(cuda), x.float().to(cuda))
    assert torch.equal(dw, dw2)  # deterministic


def test_linear_module_grads_match_torch(cuda):
    from x2gnn.layers import Linear

    torch.manual_seed(0)
    lin = Linear(128, 64).to(cuda)
    ref = torch.nn.Linear(128, 64).to(cuda)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(3, 700, 128, device=cuda)
    x1, x2 = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    g = torch.randn(3, 700, 64, device=cuda)
    (lin(x1) * g).sum().backward()
    (ref(x2) * g).sum().backward()
    for a, b in ((x1.grad, x2.grad), (lin.weight.grad, ref.weight.grad), (lin.bias.grad, ref.bias.grad)):
        np.testing.assert_allclose(a.cpu().numpy(), b.cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("R,K,N", [(21058, 128, 128), (3000, 338, 256), (2304, 128, 1), (777, 6, 128), (21058, 6, 128), (5, 6, 128),
                                   (10, 128, 128), (500, 256, 128), (130, 42, 160)])
@pytest.mark.parametrize("act", [0, 1])
@pytest.mark.parametrize("with_res", [False, True])
def test_dense_fused_vs_torch(cuda, R, K, N, act, with_res):
    from x2gnn import ops

    g = torch.Generator().manual_seed(R * 7 + K + N)
    x = torch.randn(R, K, generator=g, dtype=torch.float64)
    w = torch.randn(N, K, generator=g, dtype=torch.float64) / np.sqrt(K)
    b = torch.randn(N, generator=g, dtype=torch.float64)
    res = torch.randn(R, N, generator=g, dtype=torch.float64) if with_res else None
    up = torch.randn(R, N, generator=g, dtype=torch.float64)
    xs, ws, bs = (t.clone().requires_grad_(True) for t in (x, w, b))
    ref = xs @ ws.t() + bs
    if act:
        ref = torch.nn.functional.silu(ref)
    if with_res:
        rs = res.clone().requires_grad_(True)
        ref = ref + rs
    (ref * up).sum().backward()
    xg, wg, bg = (t.float().to(cuda).requires_grad_(True) for t in (x, w, b))
    rg = res.float().to(cuda).requires_grad_(True) if with_res else None
    y = ops.dense(xg, wg, bg, act=act, res=rg)
    (y * up.float().to(cuda)).sum().backward()
    tol = dict(rtol=1e-4, atol=1e-4 * max(1.0, np.sqrt(R / 100)))
    np.testing.assert_allclose(y.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(xg.grad.cpu().numpy(), xs.grad.numpy(), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(wg.grad.cpu().numpy(), ws.grad.numpy(), **tol)
    np.testing.assert_allclose(bg.grad.cpu().numpy(), bs.grad.numpy(), **tol)
    if with_res:
        np.testing.assert_allclose(rg.grad.cpu().numpy(), rs.grad.numpy(), rtol=1e-6, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("R,K,N,act", [(21058, 128, 128, 1), (300, 128, 128, 0), (2304, 128, 4, 1),
                                       (1000, 6, 128, 1)])
def test_dense_bwd_ex_dx_add_and_accumulate(cuda, R, K, N, act):
    """x2g_dense_bwd_ex: dx = dz w + dx_add (dx_add aliasing dx too) and X2G_ACCUM_WGRAD
    (dw += ..., db += ...) give exactly the plain backward's values plus the addend."""
    from x2gnn import _lib
    from x2gnn._lib import call, ptr, stream_ptr

    g = torch.Generator(device=cuda).manual_seed(R + K + N)
    x = torch.randn(R, K, device=cuda, generator=g)
    w = torch.randn(N, K, device=cuda, generator=g) / np.sqrt(K)
    z = torch.randn(R, N, device=cuda, generator=g)
    dy = torch.randn(R, N, device=cuda, generator=g)
    add = torch.randn(R, K, device=cuda, generator=g)
    wsb = int(_lib.load().x2g_dense_bwd_workspace(R, K, N))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=cuda)
    dx0, dw0, db0 = torch.empty(R, K, device=cuda), torch.empty(N, K, device=cuda), torch.empty(N, device=cuda)
    call("x2g_dense_bwd", ptr(dy), ptr(z), act, ptr(x), ptr(w), R, K, N, ptr(dx0), ptr(dw0), ptr(db0), ptr(ws), wsb,
         stream_ptr())
    # separate addend, accumulate into pre-filled weight-gradient buffers
    dx1 = torch.empty(R, K, device=cuda)
    dw1, db1 = torch.full((N, K), 0.5, device=cuda), torch.full((N,), -0.25, device=cuda)
    call("x2g_dense_bwd_ex", ptr(dy), ptr(z), act, ptr(x), ptr(w), R, K, N, ptr(dx1), ptr(add), ptr(dw1), ptr(db1), 1,
         ptr(ws), wsb, stream_ptr())
    # in-place: dx_add aliases dx
    dx2 = add.clone()
    dw2, db2 = torch.empty(N, K, device=cuda), torch.empty(N, device=cuda)
    call("x2g_dense_bwd_ex", ptr(dy), ptr(z), act, ptr(x), ptr(w), R, K, N, ptr(dx2), ptr(dx2), ptr(dw2), ptr(db2), 0,
         ptr(ws), wsb, stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0 + add) and torch.equal(dx2, dx0 + add)
    assert torch.equal(dw1, dw0 + 0.5) and torch.equal(db1, db0 - 0.25)
    assert torch.equal(dw2, dw0) and torch.equal(db2, db0)


@pytest.mark.gpu
@pytest.mark.parametrize("max_norm", [100.0, 0.05])
def test_flat_adam_matches_torch(cuda, max_norm):
    """x2g_clip_adam_ema (FlatAdam) vs torch clip_grad_norm_ + Adam + the reference's EMA
    (torch.optim.swa_utils.AveragedModel with avg_fn = d*avg + (1-d)*p, train_ema.py:45-47: the
    first update copies the parameters), three steps, clipping inactive (100) and active (0.05);
    each update also zeroes the gradient bucket (the trainer's folded zero_grad())."""
    from torch.optim.swa_utils import AveragedModel

    from x2gnn.dist import GradBucket
    from x2gnn.optim import FlatAdam

    g = torch.Generator(device=cuda).manual_seed(11)
    shapes = [(128, 128), (128,), (6, 128), (1,), (42, 3)]
    ref = [torch.randn(s, device=cuda, generator=g).requires_grad_(True) for s in shapes]
    mine = [r.detach().clone().requires_grad_(True) for r in ref]
    opt_ref = torch.optim.Adam(ref, lr=1e-3)
    holder = torch.nn.Module()
    holder.ps = torch.nn.ParameterList([torch.nn.Parameter(r) for r in ref])
    decay = 0.95
    ema_model = AveragedModel(holder, avg_fn=lambda avg, p, n: decay * avg + (1 - decay) * p)
    ema_ref = list(ema_model.module.ps)
    bucket = GradBucket(mine)
    opt = FlatAdam(mine, lr=1e-3, max_norm=max_norm, ema_decay=decay, bucket=bucket)
    for step in range(3):
        grads = [torch.randn(s, device=cuda, generator=g) for s in shapes]
        for r, gr in zip(ref, grads):
            r.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(ref, max_norm)
        opt_ref.step()
        ema_model.update_parameters(holder)
        if step == 0:
            bucket.zero()
        assert float(bucket.flat.abs().max()) == 0.0  # steps 1, 2: zeroed by the previous update
        for m, gr in zip(mine, grads):
            m.grad.copy_(gr)
        opt.step(zero_grads=True)  # zero_grad() folded into the update (X2G_OPT_ZERO_GRADS)
        for r, m in zip(ref, mine):
            torch.testing.assert_close(m.detach(), r.detach(), rtol=2e-6, atol=2e-7)
        for e, m in zip(ema_ref, opt.ema_params()):
            torch.testing.assert_close(m, e.detach(), rtol=2e-6, atol=2e-7)
        if step == 0:  # AveragedModel's first update is a copy of the stepped parameters
            for p, m in zip(mine, opt.ema_params()):
                assert torch.equal(m, p.detach())
    assert float(opt.steps) == 3.0


@pytest.mark.parametrize("staircase", [False, True])
def test_flat_adam_lr_schedule_matches_lambda_lr(cuda, staircase):
    """FlatAdam.set_schedule (the device-side LinearWarmupExponentialDecay) vs torch Adam driven by
    LambdaLR with the reference's lr_lambda (scheduler.py:19-26, restated here: the reference cannot
    be imported on the GPU box), scheduler.step() after every optimizer.step() as trainer.py:44-47
    does; the update is replayed from ONE captured HIP graph, so the schedule must come from the
    device step count.  Warmup 3 / decay 4 steps / rate 0.5 so 9 steps cross both regimes."""
    from x2gnn.dist import GradBucket
    from x2gnn.optim import FlatAdam

    W, DS, RATE = 3, 4, 0.5

    def lr_lambda(step):
        warmup = min(1 / W + 1 / W * step, 1)
        exponent = step / DS
        if staircase:
            exponent = int(exponent)
        return warmup * RATE ** exponent

    g = torch.Generator(device=cuda).manual_seed(12)
    shapes = [(64, 32), (32,), (5,)]
    ref = [torch.randn(s, device=cuda, generator=g).requires_grad_(True) for s in shapes]
    mine = [r.detach().clone().requires_grad_(True) for r in ref]
    opt_ref = torch.optim.Adam(ref, lr=1e-2)
    sched = torch.optim.lr_scheduler.LambdaLR(opt_ref, lr_lambda)
    bucket = GradBucket(mine)
    opt = FlatAdam(mine, lr=1e-2, max_norm=100.0, ema_decay=None, bucket=bucket)
    opt.set_schedule(W, DS, RATE, staircase=staircase)
    grads = [[torch.randn(s, device=cuda, generator=g) for s in shapes] for _ in range(9)]
    stage = [torch.zeros(s, device=cuda) for s in shapes]
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        for m, st in zip(mine, stage):
            m.grad.copy_(st)
        opt.step()
    for step in range(9):
        lr_used = opt_ref.param_groups[0]["lr"]
        for r, gr in zip(ref, grads[step]):
            r.grad = gr.clone()
        torch.nn.utils.clip_grad_norm_(ref, 100.0)
        opt_ref.step()
        sched.step()
        for st, gr in zip(stage, grads[step]):
            st.copy_(gr)
        graph.replay()
        torch.cuda.synchronize()
        assert abs(float(opt.lr) - lr_used) <= 1e-7 * lr_used, (step, float(opt.lr), lr_used)
        for r, m in zip(ref, mine):
            torch.testing.assert_close(m.detach(), r.detach(), rtol=2e-6, atol=2e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("T,out_dim", [(194060, 128), (1000, 128), (37, 128), (0, 128), (1000, 256), (37, 256),
                                       (1000, 64), (37, 32)])
def test_sbf_project_vs_torch(cuda, T, out_dim):
    """x2g_sbf_project: the wave-independent MFMA kernel (out_dim 128 / 64) and the VALU path
    (out_dim 256, e.g. xgnn_poly's default in_channels=256, xgnn.py:16; and 32).  T = 37 makes 37*42
    floats, not a multiple of 4: the last 16-byte chunk is partial."""
    from x2gnn._lib import call, ptr, stream_ptr

    g = torch.Generator(device=cuda).manual_seed(T + 5 + out_dim)
    sbf = torch.randn(T, 42, device=cuda, generator=g)
    w = torch.randn(out_dim, 42, device=cuda, generator=g) / 6.5
    b = torch.randn(out_dim, device=cuda, generator=g)
    ref = (sbf.double() @ w.double().t() + b.double()).float()
    out = torch.full((T, out_dim), float("nan"), device=cuda)
    call("x2g_sbf_project", ptr(sbf), T, 42, ptr(w), ptr(b), out_dim, ptr(out), stream_ptr())
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("T,out_dim,n", [(194060, 128, 4), (37, 128, 3), (1000, 64, 2), (0, 128, 4)])
def test_sbf_project_batch_equals_per_layer(cuda, T, out_dim, n):
    """x2g_sbf_project_batch (every layer's lin_sbf in one launch, layer = blockIdx.y; out_dim 64 takes the
    per-layer fallback) == x2g_sbf_project per layer, bit for bit, and == fp64 torch to rounding."""
    import ctypes

    from x2gnn._lib import call, ptr, stream_ptr

    g = torch.Generator(device=cuda).manual_seed(T + n)
    sbf = torch.randn(T, 42, device=cuda, generator=g)
    ws = [torch.randn(out_dim, 42, device=cuda, generator=g) / 6.5 for _ in range(n)]
    bs = [torch.randn(out_dim, device=cuda, generator=g) for _ in range(n)]
    outs = [torch.full((T, out_dim), float("nan"), device=cuda) for _ in range(n)]
    P = ctypes.c_void_p * n
    call("x2g_sbf_project_batch", ptr(sbf), T, 42, P(*[w.data_ptr() for w in ws]), P(*[b.data_ptr() for b in bs]), n,
         out_dim, P(*[o.data_ptr() for o in outs]), stream_ptr())
    for w, b, o in zip(ws, bs, outs):
        one = torch.full((T, out_dim), float("nan"), device=cuda)
        call("x2g_sbf_project", ptr(sbf), T, 42, ptr(w), ptr(b), out_dim, ptr(one), stream_ptr())
        assert torch.equal(o, one)
        torch.testing.assert_close(o, (sbf.double() @ w.double().t() + b.double()).float(), rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_sbf_project_rows_independent_of_nonfinite_neighbours(cuda):
    """A non-finite sbf row poisons only its own projection (the reference's lin_sbf is row-wise):
    the narrow-K kernel's LDS span has row stride K, so a row's pad columns alias the next row."""
    from x2gnn._lib import call, ptr, stream_ptr

    T = 200
    g = torch.Generator(device=cuda).manual_seed(3)
    sbf = torch.randn(T, 42, device=cuda, generator=g)
    bad = [5, 64, 65, 127, 199]  # inside a tile, first rows of a pair, the last row
    sbf[bad[0], 0] = float("inf")
    sbf[bad[1], :4] = float("nan")
    sbf[bad[2], 1] = float("-inf")
    sbf[bad[3], 0] = float("nan")
    sbf[bad[4], 3] = float("inf")
    w = torch.randn(128, 42, device=cuda, generator=g) / 6.5
    b = torch.randn(128, device=cuda, generator=g)
    out = torch.empty(T, 128, device=cuda)
    call("x2g_sbf_project", ptr(sbf), T, 42, ptr(w), ptr(b), 128, ptr(out), stream_ptr())
    torch.cuda.synchronize()
    good = torch.ones(T, dtype=torch.bool)
    good[bad] = False
    assert torch.isfinite(out[good.to(cuda)]).all()
    ref = (sbf.double() @ w.double().t() + b.double()).float()
    torch.testing.assert_close(out[good.to(cuda)], ref[good.to(cuda)], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("R,K", [(5000, 42), (333, 10), (64, 42), (65, 126), (37, 42), (1, 42), (63, 6 * 7 + 1)])
def test_dense_narrow_k_vs_torch(cuda, R, K):
    from x2gnn import ops

    g = torch.Generator(device=cuda).manual_seed(R + K)
    x = torch.randn(R, K, device=cuda, generator=g)
    w = torch.randn(128, K, device=cuda, generator=g) / np.sqrt(K)
    b = torch.randn(128, device=cuda, generator=g)
    res = torch.randn(R, 128, device=cuda, generator=g)
    y = ops.dense(x, w, b, act=ops.ACT_SILU, res=res)
    ref = torch.nn.functional.silu(x.double() @ w.double().t() + b.double()) + res.double()
    torch.testing.assert_close(y.double(), ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("E", [0, 1, 3000])
def test_edge_basis_vs_torch(cuda, E):
    """x2g_edge_basis (dist, envelope, trainable radial basis, Bessel terms) and its frequency
    gradient against the torch formulas (xgnn.py:49-53, radial_basis_layer.py:36-40)."""
    from x2gnn import ops
    from x2gnn.layers import RadialBasis, poly_envelop

    g = torch.Generator().manual_seed(5)
    n_atoms = 40
    pos = (torch.rand(n_atoms, 3, generator=g) * 4.0).to(cuda)
    src = torch.randint(0, n_atoms, (E,), generator=g)
    dst = (src + torch.randint(1, n_atoms, (E,), generator=g)) % n_atoms
    lg = ops.LineGraph.__new__(ops.LineGraph)
    lg.E, lg.edge_src, lg.edge_dst = E, src.to(torch.int32).to(cuda), dst.to(torch.int32).to(cuda)
    rb = RadialBasis(embedding_size=6, cutoff=5.0).to(cuda)
    with torch.no_grad():
        rb.frequencies.mul_(1.0 + 0.1 * torch.rand(6, generator=g).to(cuda))
    dist, env, rbf, bes = ops.edge_basis(pos, lg, rb.frequencies, 5.0)
    d_ref = (pos[src.to(cuda)] - pos[dst.to(cuda)]).norm(dim=1)
    env_ref = poly_envelop(5.0, 5)(d_ref)
    torch.testing.assert_close(dist, d_ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(env, env_ref, rtol=2e-5, atol=1e-5)
    f2 = rb.frequencies.detach().clone().requires_grad_(True)
    rbf_ref = torch.sin(f2 * (d_ref * 0.2).unsqueeze(-1)) * env_ref.unsqueeze(1)
    torch.testing.assert_close(rbf, rbf_ref, rtol=5e-5, atol=5e-5)
    torch.testing.assert_close(bes, ops.bessel_env(dist, 5.0), rtol=1e-6, atol=1e-6)
    up = torch.randn(E, 6, generator=g).to(cuda)
    (rbf * up).sum().backward()
    (rbf_ref * up).sum().backward()
    if E == 0:
        assert rb.frequencies.grad is None or float(rb.frequencies.grad.abs().max()) == 0.0
    else:
        torch.testing.assert_close(rb.frequencies.grad, f2.grad, rtol=2e-4, atol=2e-4)


def _gate_inputs(cuda, rows, D, R, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(rows, D, generator=g).to(cuda)
    rbf = torch.randn(rows, R, generator=g).to(cuda)
    w = (0.3 * torch.randn(D, R, generator=g)).to(cuda)
    b = (0.1 * torch.randn(D, generator=g)).to(cuda)
    return x, rbf, w, b


@pytest.mark.parametrize("rows,D,R,bias", [(1, 128, 6, True), (2049, 128, 6, False), (777, 64, 3, True),
                                           (300, 256, 8, True), (21058, 128, 6, False)])
def test_rbf_gate_vs_torch(cuda, rows, D, R, bias):
    """x2g_rbf_gate_fwd/bwd: x * (W rbf + b) and all four gradients vs torch autograd."""
    from x2gnn import _lib, ops
    from x2gnn._lib import call, ptr, stream_ptr

    x, rbf, w, b = _gate_inputs(cuda, rows, D, R, rows + D)
    b = b if bias else None
    out = torch.empty_like(x)
    call("x2g_rbf_gate_fwd", ptr(x), ptr(rbf), ptr(w), ptr(b), rows, D, R, ptr(out), stream_ptr())
    xr, rr, wr = (t.clone().requires_grad_(True) for t in (x, rbf, w))
    br = b.clone().requires_grad_(True) if bias else None
    f = torch.nn.functional.linear(rr, wr, br)
    ref = xr * f
    torch.testing.assert_close(out, ref.detach(), rtol=1e-5, atol=1e-5)
    gy = torch.randn(rows, D, device=cuda)
    ref.backward(gy)
    add = torch.randn(rows, D, device=cuda)
    dx, drbf, dw, db = ops._gate_bwd(gy, None, x, rbf, w, b, None, None, True, True, dx_add=add)
    torch.testing.assert_close(dx, xr.grad + add, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(drbf, rr.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dw, wr.grad, rtol=1e-4, atol=1e-3)
    if bias:
        torch.testing.assert_close(db, br.grad, rtol=1e-4, atol=1e-3)
    # accumulate into existing buffers (X2G_ACCUM_WGRAD)
    dw2, db2 = torch.ones_like(w), (torch.ones_like(b) if bias else None)
    ws_bytes = int(_lib.load().x2g_rbf_gate_bwd_workspace(rows, D, R))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    call("x2g_rbf_gate_bwd", ptr(gy), None, ptr(x), ptr(rbf), ptr(w), ptr(b), rows, D, R, None, None, None, ptr(dw2),
         ptr(db2), 1, ptr(ws), ws_bytes, stream_ptr())
    torch.testing.assert_close(dw2, wr.grad + 1, rtol=1e-4, atol=1e-3)


def test_rbf_gate_bwd_beyond_32bit_offsets(cuda):
    """The gate backward at rows x D x 4 >= 2^31 bytes (4.2M rows at D = 128): without the optional
    operands that take 32-bit buffer offsets it runs (dx, dW, db vs an fp64 reduction); with dx_add it
    refuses (X2G_EUNSUPPORTED) instead of reading wrapped offsets."""
    from x2gnn import _lib
    from x2gnn._lib import call, ptr, stream_ptr

    rows, D, R = (1 << 31) // (128 * 4) + 96, 128, 6
    g = torch.Generator(device=cuda).manual_seed(5)
    x = torch.randn(rows, D, device=cuda, generator=g)
    gy = torch.randn(rows, D, device=cuda, generator=g)
    rbf = torch.randn(rows, R, device=cuda, generator=g)
    w = 0.3 * torch.randn(D, R, device=cuda, generator=g)
    b = 0.1 * torch.randn(D, device=cuda, generator=g)
    dx = torch.empty_like(x)
    dw, db = torch.empty_like(w), torch.empty_like(b)
    ws_bytes = int(_lib.load().x2g_rbf_gate_bwd_workspace(rows, D, R))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    call("x2g_rbf_gate_bwd", ptr(gy), None, ptr(x), ptr(rbf), ptr(w), ptr(b), rows, D, R, ptr(dx), None, None,
         ptr(dw), ptr(db), 0, ptr(ws), ws_bytes, stream_ptr())
    tail = slice(rows - 5000, rows)
    want = gy[tail] * torch.nn.functional.linear(rbf[tail], w, b)
    torch.testing.assert_close(dx[tail], want, rtol=1e-5, atol=1e-5)
    gx = (gy * x).double()
    ref_w = gx.t() @ rbf.double()
    ref_b = gx.sum(0)
    del gx
    scale = float(ref_w.abs().max())
    assert float((dw.double() - ref_w).abs().max()) <= 1e-5 * scale + 1e-3
    assert float((db.double() - ref_b).abs().max()) <= 1e-5 * float(ref_b.abs().max()) + 1e-3
    add = torch.zeros(8, device=cuda)  # present (its size is not what is checked)
    with pytest.raises(RuntimeError):
        call("x2g_rbf_gate_bwd", ptr(gy), None, ptr(x), ptr(rbf), ptr(w), ptr(b), rows, D, R, ptr(dx), ptr(add),
             None, ptr(dw), ptr(db), 0, ptr(ws), ws_bytes, stream_ptr())


def test_rbf_pool_vs_torch(cuda):
    """x2g_rbf_pool_fwd + the owner-indexed backward: segment sums of x * (W rbf + b) over
    ragged (and empty) segments vs torch index_add + autograd."""
    from x2gnn import ops

    rng = np.random.default_rng(3)
    rowptr = _rowptr_with_empties(rng, 300, 17)
    rows = int(rowptr[-1])
    owner = torch.from_numpy(np.repeat(np.arange(300), np.diff(rowptr))).to(cuda)
    x, rbf, w, b = _gate_inputs(cuda, rows, 128, 6, 9)
    w.requires_grad_(True)
    b.requires_grad_(True)
    xr, rr = x.clone().requires_grad_(True), rbf.clone().requires_grad_(True)
    out = ops.rbf_pool(xr, rr, w, b, owner, torch.from_numpy(rowptr).to(cuda), 300)
    xq, rq = x.clone().requires_grad_(True), rbf.clone().requires_grad_(True)
    wq, bq = w.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    ref = torch.zeros(300, 128, device=cuda).index_add(0, owner, xq * torch.nn.functional.linear(rq, wq, bq))
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-4)
    gy = torch.randn(300, 128, device=cuda)
    out.backward(gy)
    ref.backward(gy)
    torch.testing.assert_close(xr.grad, xq.grad, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(rr.grad, rq.grad, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(w.grad, wq.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(b.grad, bq.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("n_jobs,D,bias", [(5, 128, True), (2, 64, False), (8, 256, True)])
def test_rbf_pool_batch_vs_torch(cuda, n_jobs, D, bias):
    """ops.rbf_pool_batch (x2g_rbf_pool_fwd_batch / x2g_rbf_gate_bwd_batch: several readouts'
    pools in one launch each way, the basis gradient summed over jobs) vs torch index_add +
    autograd over ragged and empty segments, with and without a gradient bucket + deferred slab
    sums; the forward is bitwise the single-job kernel's."""
    from x2gnn import ops
    from x2gnn.dist import GradBucket

    rng = np.random.default_rng(n_jobs + D)
    rowptr = _rowptr_with_empties(rng, 300, 17)
    rows = int(rowptr[-1])
    owner = torch.from_numpy(np.repeat(np.arange(300), np.diff(rowptr))).to(cuda)
    rp = torch.from_numpy(rowptr).to(cuda)
    rbf = torch.randn(rows, 6, device=cuda)
    xs = [torch.randn(rows, D, device=cuda) for _ in range(n_jobs)]
    lins = [torch.nn.Linear(6, D, bias=bias).to(cuda) for _ in range(n_jobs)]
    gys = [torch.randn(300, D, device=cuda) for _ in range(n_jobs)]
    for bucket in (False, True):
        xr = [x.clone().requires_grad_(True) for x in xs]
        rr = rbf.clone().requires_grad_(True)
        for m in lins:
            m.zero_grad(set_to_none=True)
        bk = GradBucket([p for m in lins for p in m.parameters()]) if bucket else None
        if bk is not None:
            bk.zero()
        outs = ops.rbf_pool_batch(xr, rr, [m.weight for m in lins], [m.bias for m in lins], owner, rp, 300)
        for j in range(n_jobs):
            single = ops.rbf_pool(xs[j], rbf, lins[j].weight.detach(), None if not bias else lins[j].bias.detach(),
                                  owner, rp, 300)
            assert torch.equal(outs[j].detach(), single)
        with ops.deferred_wgrad():
            torch.autograd.backward(outs, gys)
        xq = [x.clone().requires_grad_(True) for x in xs]
        rq = rbf.clone().requires_grad_(True)
        ps = [(m.weight.detach().clone().requires_grad_(True),
               m.bias.detach().clone().requires_grad_(True) if bias else None) for m in lins]
        refs = [torch.zeros(300, D, device=cuda).index_add(0, owner, xq[j] * torch.nn.functional.linear(rq, *ps[j]))
                for j in range(n_jobs)]
        torch.autograd.backward(refs, gys)
        for j in range(n_jobs):
            torch.testing.assert_close(outs[j], refs[j], rtol=1e-5, atol=1e-4)
            torch.testing.assert_close(xr[j].grad, xq[j].grad, rtol=1e-5, atol=1e-5)
            torch.testing.assert_close(lins[j].weight.grad, ps[j][0].grad, rtol=1e-4, atol=1e-3)
            if bias:
                torch.testing.assert_close(lins[j].bias.grad, ps[j][1].grad, rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(rr.grad, rq.grad, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("R,D,K", [(0, 128, 10), (1, 128, 10), (21058, 128, 10), (999, 64, 16), (5000, 12, 3)])
def test_keyed_row_sum_vs_torch(cuda, R, D, K):
    """x2g_keyed_row_sum (gradient of a per-element table gather) vs index_add, and bitwise repeatable."""
    from x2gnn import ops

    g = torch.Generator().manual_seed(R + D)
    src = torch.randn(R, D, generator=g).to(cuda)
    key = torch.randint(0, K, (R,), generator=g).to(torch.int32).to(cuda)
    out = ops.keyed_row_sum(src, key, K)
    # fp64 reference: index_add in fp32 is itself order-dependent (atomics); the bound is fp32
    # summation error, a few ulp of the bucket's sum of magnitudes
    ref = torch.zeros(K, D, device=cuda, dtype=torch.float64).index_add_(0, key.long(), src.double())
    mag = torch.zeros(K, D, device=cuda, dtype=torch.float64).index_add_(0, key.long(), src.double().abs())
    assert bool(((out.double() - ref).abs() <= 1e-6 * mag + 1e-6).all())
    assert torch.equal(out, ops.keyed_row_sum(src, key, K))


@pytest.mark.parametrize("max_norm", [None, 3.0, 0.5])
def test_embedding_table_vs_torch(cuda, max_norm):
    """x2g_embedding_table (in-place renorm of the used rows, per-element rows) and its backward
    (scale_grad_by_freq, padding row) vs nn.Embedding on the same atoms."""
    from x2gnn import ops

    g = torch.Generator().manual_seed(11)
    z = torch.tensor([1, 6, 6, 8, 1, 1, 7, 0, 6, 1], dtype=torch.int64)
    ref = torch.nn.Embedding(10, 32, padding_idx=0, max_norm=max_norm, scale_grad_by_freq=True).to(cuda)
    with torch.no_grad():
        ref.weight.copy_(torch.randn(10, 32, generator=g).to(cuda))
    w = torch.nn.Parameter(ref.weight.detach().clone())
    table = ops.embedding_table(w, z.to(cuda), max_norm, 0, True)
    out = ref(z.to(cuda))
    torch.testing.assert_close(w.detach(), ref.weight.detach(), rtol=1e-6, atol=1e-7)  # same in-place renorm
    torch.testing.assert_close(table[z.to(cuda)], out.detach(), rtol=1e-6, atol=1e-7)
    up = torch.randn(10, 32, generator=g).to(cuda)
    out.backward(up)
    # the per-atom upstream gradient summed per element is what the table receives
    gt = torch.zeros(10, 32, device=cuda).index_add_(0, z.to(cuda), up)
    table.backward(gt)
    torch.testing.assert_close(w.grad, ref.weight.grad, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("R,G", [(2304, 5), (1, 1), (37, 8), (128, 5)])
def test_readout_mlps_batched_vs_separate(cuda, R, G):
    """ops.readout_mlps (batched dense fwd/bwd + the fused Linear(D,1) head summed over readouts)
    equals sum_g run_mlp(mlp_g, feat_g) in value and in every gradient."""
    from x2gnn import ops
    from x2gnn.layers import _mlp, run_mlp

    torch.manual_seed(R + G)
    mlps = [_mlp(128, 1, 3).to(cuda) for _ in range(G)]
    mlps_ref = [_mlp(128, 1, 3).to(cuda) for _ in range(G)]
    for a, b in zip(mlps, mlps_ref):
        b.load_state_dict(a.state_dict())
    feats = [torch.randn(R, 128, device=cuda, requires_grad=True) for _ in range(G)]
    feats_ref = [f.detach().clone().requires_grad_(True) for f in feats]
    assert ops.readout_mlps_supported(feats, mlps)
    out = ops.readout_mlps(feats, mlps)
    ref = None
    for m, f in zip(mlps_ref, feats_ref):
        r = run_mlp(m, f)
        ref = r if ref is None else ref + r
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    up = torch.randn(R, 1, device=cuda)
    out.backward(up)
    ref.backward(up)
    for f, fr in zip(feats, feats_ref):
        torch.testing.assert_close(f.grad, fr.grad, rtol=1e-5, atol=1e-5)
    for a, b in zip(mlps, mlps_ref):
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-4, msg=n)


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,G", [([18] * 128, 5), ([1], 1), ([5, 0, 40, 1, 3], 3), ([300, 2, 61], 8)])
def test_readout_heads_pooled_vs_pool_after(cuda, sizes, G):
    """ops.readout_mlps(pool=(mol_ptr, B)): the heads with the global add pool fused (x2g_readout_head_pool_*,
    model.py:53) equal the per-row heads followed by ops.segment_sum — values, every feature gradient and
    every parameter gradient (fp32 reassociation: the pooled sum runs in a different order); segments of
    0, 1 and > 256 rows."""
    from x2gnn import ops
    from x2gnn.layers import _mlp

    R = sum(sizes)
    torch.manual_seed(R + G)
    mlps = [_mlp(128, 1, 3).to(cuda) for _ in range(G)]
    mlps_ref = [_mlp(128, 1, 3).to(cuda) for _ in range(G)]
    for a, b in zip(mlps, mlps_ref):
        b.load_state_dict(a.state_dict())
    ptr = torch.tensor([0] + list(torch.tensor(sizes).cumsum(0)), dtype=torch.int32, device=cuda)
    feats = [torch.randn(R, 128, device=cuda, requires_grad=True) for _ in range(G)]
    feats_ref = [f.detach().clone().requires_grad_(True) for f in feats]
    out = ops.readout_mlps(feats, mlps, pool=(ptr, len(sizes)))
    ref = ops.segment_sum(ops.readout_mlps(feats_ref, mlps_ref), ptr, len(sizes))
    assert out.shape == ref.shape == (len(sizes), 1)
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-5)
    up = torch.randn(len(sizes), 1, device=cuda)
    out.backward(up)
    ref.backward(up)
    for f, fr in zip(feats, feats_ref):
        torch.testing.assert_close(f.grad, fr.grad, rtol=1e-5, atol=1e-6)
    for a, b in zip(mlps, mlps_ref):
        for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
            torch.testing.assert_close(p.grad, q.grad, rtol=1e-4, atol=1e-5, msg=n)


@pytest.mark.parametrize("R,D", [(1, 128), (33, 128), (21058, 128), (500, 64), (77, 12)])
def test_fused_residual_layer_vs_torch(cuda, R, D):
    """x2g_residual_fwd (both GEMMs of a ResidualLayer in one kernel) + the layer's backward vs
    torch: y = x + SiLU(W1 SiLU(W0 x + b0) + b1)."""
    from x2gnn.layers import ResidualLayer

    torch.manual_seed(R + D)
    layer = ResidualLayer(D).to(cuda)
    x = torch.randn(R, D, device=cuda, requires_grad=True)
    y = layer(x)
    xr = x.detach().clone().requires_grad_(True)
    F = torch.nn.functional
    ref = xr + F.silu(F.linear(F.silu(F.linear(xr, layer.lin0.weight, layer.lin0.bias)), layer.lin1.weight,
                               layer.lin1.bias))
    torch.testing.assert_close(y, ref, rtol=2e-5, atol=2e-5)
    up = torch.randn(R, D, device=cuda)
    y.backward(up)
    gw = [p.grad.clone() for p in layer.parameters()]
    for p in layer.parameters():
        p.grad = None
    ref.backward(up)
    torch.testing.assert_close(x.grad, xr.grad, rtol=1e-4, atol=1e-4)
    for a, p in zip(gw, layer.parameters()):
        torch.testing.assert_close(a, p.grad, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("E,D", [(0, 128), (1, 128), (31, 64), (21058, 128), (5000, 32)])
def test_sbf_radial_wgrad_vs_fp64(cuda, E, D):
    """x2g_sbf_radial_wgrad: dW[c, 6l+n] = sum_s R[s, 6l+n] G[s, l, c], db[c] = sum_s G[s, 7, c]."""
    from x2gnn import ops

    g = torch.Generator().manual_seed(E + D)
    G = torch.randn(E, 8, D, generator=g)
    R = torch.randn(E, 42, generator=g)
    dw, db = ops.sbf_radial_wgrad(G.to(cuda), R.to(cuda))
    ref_w = torch.einsum("sld,sln->dln", G[:, :7].double(), R.view(E, 7, 6).double()).reshape(D, 42)
    ref_b = G[:, 7].double().sum(0)
    mag = torch.einsum("sld,sln->dln", G[:, :7].double().abs(), R.view(E, 7, 6).double().abs()).reshape(D, 42)
    assert bool(((dw.cpu().double() - ref_w).abs() <= 1e-6 * mag + 1e-6).all())
    assert bool(((db.cpu().double() - ref_b).abs() <= 1e-6 * G[:, 7].double().abs().sum(0) + 1e-6).all())
    dw2, _ = ops.sbf_radial_wgrad(G.to(cuda), R.to(cuda))
    assert torch.equal(dw, dw2)


def _chain_ref(x, res, ws, bs, flags):
    """fp64 torch restatement of x2g_chain_fwd (include/x2g.h: row chains)."""
    from x2gnn import ops

    held = None
    cur = x
    for w, b, f in zip(ws, bs, flags):
        if f & ops.CHAIN_RES_EXT:
            held = res
        if f & ops.CHAIN_HOLD:
            held = cur
        z = cur @ w.t() + (b if b is not None else 0.0)
        y = torch.nn.functional.silu(z) if f & ops.CHAIN_SILU else z
        if f & (ops.CHAIN_RES_HELD | ops.CHAIN_RES_EXT):
            y = y + held
        cur = y
    return cur


@pytest.mark.gpu
@pytest.mark.parametrize("R", [21058, 1000, 37, 16, 1])
@pytest.mark.parametrize("kind", ["trunk", "plain", "residual"])
def test_row_chain_fwd_bwd_vs_torch(cuda, R, kind):
    """x2g_chain_fwd / x2g_chain_bwd / x2g_wgrad_batched (ops.row_chain) against fp64 torch
    autograd: the trunk tail of model.py:47-50 (7 stages), a plain Linear without activation,
    and one ResidualLayer; ragged tiles (R % 16 != 0) and fewer rows than one tile."""
    from x2gnn import ops

    S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
    flags = {"trunk": [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH], "plain": [0],
             "residual": [S | H, S | RH]}[kind]
    n = len(flags)
    g = torch.Generator(device=cuda).manual_seed(R + n)
    lins = [torch.nn.Linear(128, 128, bias=(i != 1 or kind != "trunk")).to(cuda) for i in range(n)]
    with torch.no_grad():
        for m in lins:
            m.weight.copy_(torch.randn(128, 128, device=cuda, generator=g) / 11.3)
            if m.bias is not None:
                m.bias.copy_(torch.randn(128, device=cuda, generator=g) * 0.1)
    x = torch.randn(R, 128, device=cuda, generator=g).requires_grad_(True)
    res = torch.randn(R, 128, device=cuda, generator=g).requires_grad_(True) if kind == "trunk" else None
    y = ops.row_chain(x, res, lins, flags)
    dy = torch.randn(R, 128, device=cuda, generator=g)
    y.backward(dy)
    xd = x.detach().double().requires_grad_(True)
    rd = res.detach().double().requires_grad_(True) if res is not None else None
    wd = [m.weight.detach().double().requires_grad_(True) for m in lins]
    bd = [m.bias.detach().double().requires_grad_(True) if m.bias is not None else None for m in lins]
    yr = _chain_ref(xd, rd, wd, bd, flags)
    yr.backward(dy.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.double(), xd.grad, rtol=1e-5, atol=1e-5)
    if res is not None:
        torch.testing.assert_close(res.grad.double(), rd.grad, rtol=1e-5, atol=1e-5)
    for m, w, b in zip(lins, wd, bd):
        scale = float(w.grad.abs().max())
        assert float((m.weight.grad.double() - w.grad).abs().max()) <= 2e-5 * scale + 1e-6
        if b is not None:
            assert float((m.bias.grad.double() - b.grad).abs().max()) <= 2e-5 * float(b.grad.abs().max()) + 1e-6


def _graph_ln_ref(x, rowptr, eps):
    """PyG LayerNorm(mode='graph', affine=False) per row segment (two-pass, biased variance)."""
    out = torch.empty_like(x)
    rp = rowptr.tolist()
    for g in range(len(rp) - 1):
        a, b = rp[g], rp[g + 1]
        if b > a:
            xs = x[a:b]
            xc = xs - xs.mean()
            out[a:b] = xc / torch.sqrt((xc * xc).mean() + eps)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", ["qm9", "ragged"])
def test_row_chain_fused_graph_layernorm(cuda, sizes):
    """ops.row_chain(x, ..., ln=...) (x2g_chain_fwd_ln: the graph LayerNorm of model.py:46 applied
    while staging, from per-row (mean, M2) statistics) == LayerNorm then row_chain, forward and every
    gradient, against fp64 torch; segments of 1..400 rows (chunks holding many molecules, molecules
    spanning several chunks) and empty segments; the row statistics as x2g_sbf_attention_fwd_stats
    writes them."""
    from x2gnn import ops

    g = torch.Generator(device="cpu").manual_seed(7)
    if sizes == "qm9":
        counts = [165] * 128
    else:
        counts = [int(c) for c in torch.randint(0, 40, (60,), generator=g)] + [0, 400, 1, 0, 2, 257]
    rowptr = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32)
    R, G, eps = int(rowptr[-1]), len(counts), 1e-8
    S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
    flags = [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH]
    gd = torch.Generator(device=cuda).manual_seed(R)
    lins = [torch.nn.Linear(128, 128).to(cuda) for _ in flags]
    with torch.no_grad():
        for m in lins:
            m.weight.copy_(torch.randn(128, 128, device=cuda, generator=gd) / 11.3)
            m.bias.copy_(torch.randn(128, device=cuda, generator=gd) * 0.1)
    x = (torch.randn(R, 128, device=cuda, generator=gd) * 2.0 + 0.7).requires_grad_(True)
    res = torch.randn(R, 128, device=cuda, generator=gd).requires_grad_(True)
    xd = x.detach()
    mu_r = xd.mean(1)
    stats = torch.stack([mu_r, ((xd - mu_r[:, None]) ** 2).sum(1)], 1).contiguous()
    y = ops.row_chain(x, res, lins, flags, ln=(stats, rowptr.to(cuda), G, eps))
    dy = torch.randn(R, 128, device=cuda, generator=gd)
    y.backward(dy)
    x64 = x.detach().double().requires_grad_(True)
    r64 = res.detach().double().requires_grad_(True)
    wd = [m.weight.detach().double().requires_grad_(True) for m in lins]
    bd = [m.bias.detach().double().requires_grad_(True) for m in lins]
    yr = _chain_ref(_graph_ln_ref(x64, rowptr, eps), r64, wd, bd, flags)
    yr.backward(dy.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-5, atol=1e-5 * float(x64.grad.abs().max()))
    torch.testing.assert_close(res.grad.double(), r64.grad, rtol=1e-5, atol=1e-5)
    for m, w, b in zip(lins, wd, bd):
        assert float((m.weight.grad.double() - w.grad).abs().max()) <= 2e-5 * float(w.grad.abs().max()) + 1e-6
        assert float((m.bias.grad.double() - b.grad).abs().max()) <= 2e-5 * float(b.grad.abs().max()) + 1e-6


@pytest.mark.gpu
def test_attention_row_stats(cuda):
    """x2g_sbf_attention_fwd_stats: the same outputs as x2g_sbf_attention_fwd (bitwise) plus per-row
    (mean, sum of squared deviations) of out, vs torch."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr

    z = golden("triplets.npz")
    lg = _lg(z["s160_edge_index"], int(z["s160_num_nodes"]), z["s160_trip"].shape[1], cuda)
    E, T, H, C = lg.E, lg.T, 16, 8
    D = H * C
    gd = torch.Generator(device=cuda).manual_seed(5)
    q, k, v, skip = (torch.randn(E, D, device=cuda, generator=gd) for _ in range(4))
    table = torch.randn(10, D, device=cuda, generator=gd)
    erow = torch.randint(0, 10, (E,), device=cuda, generator=gd).to(torch.int32)
    sp = torch.randn(T, D, device=cuda, generator=gd)
    outs = []
    for stats in (None, torch.empty(E, 2, device=cuda)):
        out, alpha = torch.empty(E, D, device=cuda), torch.empty(T, H, device=cuda)
        smax, sden = torch.empty(E, H, device=cuda), torch.empty(E, H, device=cuda)
        name = "x2g_sbf_attention_fwd" if stats is None else "x2g_sbf_attention_fwd_stats"
        call(name, ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(erow), ops.EDGE_PER_DST, ptr(sp), None, None,
             ptr(lg.trip_rowptr), ptr(lg.trip_src), E, T, H, C, D, ptr(out), ptr(alpha), ptr(smax), ptr(sden),
             *((ptr(stats),) if stats is not None else ()), stream_ptr())
        outs.append((out, alpha, stats))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    o = outs[1][0].double()
    mu = o.mean(1)
    torch.testing.assert_close(outs[1][2][:, 0].double(), mu, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(outs[1][2][:, 1].double(), ((o - mu[:, None]) ** 2).sum(1), rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_row_chain_rejects_bad_programs(cuda):
    """RES_HELD without a HOLD, two RES_EXT stages, a HOLD..RES_HELD pair spanning the RES_EXT
    stage, and a width other than 128 are refused at the ABI (no kernel runs)."""
    from x2gnn import _lib, ops
    from x2gnn._lib import ptr, stream_ptr

    lib = _lib.load()
    R = 64
    x = torch.randn(R, 128, device=cuda)
    w = torch.randn(128, 128, device=cuda)
    ys = [torch.empty(R, 128, device=cuda) for _ in range(3)]
    S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT

    def run(flags, dim=128):
        st = (ops.ChainStage * len(flags))(*[ops.ChainStage(w.data_ptr(), None, None, ys[i].data_ptr(), None, f)
                                              for i, f in enumerate(flags)])
        return lib.x2g_chain_fwd(ptr(x), ptr(x), st, len(flags), R, dim, None, stream_ptr())

    assert run([S | RH]) != 0
    assert run([S | RE, S | RE]) != 0
    assert run([S | H, S | RE, S | RH]) != 0
    assert run([S | H, S | RH], dim=64) != 0
    assert run([S | H, S | RH]) == 0
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_model_chain_matches_layerwise_path(cuda, monkeypatch):
    """xgnn_poly at config width with the row-chain trunk tail (default) vs the layer-by-layer
    kernels (ops._CHAIN off): energies and every parameter gradient agree to fp32 rounding."""
    import x2gnn
    from x2gnn import ops
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    from weights import load_seeded

    cfg = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)
    b = collate(synthetic_molecules(16, "S160", seed=31)).to(cuda)
    out = []
    for on in (True, False):
        monkeypatch.setattr(ops, "_CHAIN", on)
        m = x2gnn.xgnn_poly(device="cuda", **cfg)
        load_seeded(m, 3)
        m = m.to(cuda)
        res = m(b)
        torch.nn.functional.smooth_l1_loss(res, b.y).backward()
        out.append((res.detach(), {k: p.grad.detach().clone() for k, p in m.named_parameters() if p.grad is not None}))
    (r1, g1), (r0, g0) = out
    torch.testing.assert_close(r1, r0, rtol=1e-5, atol=1e-5)
    assert g1.keys() == g0.keys()
    for k in g1:
        scale = float(g0[k].abs().max())
        assert float((g1[k] - g0[k]).abs().max()) <= 1e-4 * scale + 1e-7, k


@pytest.mark.gpu
@pytest.mark.parametrize("R", [3000, 21])
def test_row_chain_bwd_with_and_without_transposed_weights(cuda, R):
    """x2g_chain_bwd reads each stage's weight slice from x2g_chain_fwd's W^T output when given
    (contiguous loads) or transposes W itself: both give the same bits; W^T equals w.t()."""
    from x2gnn._lib import call, ptr, stream_ptr
    from x2gnn import ops

    S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
    flags = [S | H, S | RH, S | RE, S | H, S | RH]
    n = len(flags)
    g = torch.Generator(device=cuda).manual_seed(R)
    W = [torch.randn(128, 128, device=cuda, generator=g) / 11.3 for _ in range(n)]
    B = [torch.randn(128, device=cuda, generator=g) * 0.1 for _ in range(n)]
    x = torch.randn(R, 128, device=cuda, generator=g)
    res = torch.randn(R, 128, device=cuda, generator=g)
    Z = [torch.empty(R, 128, device=cuda) for _ in range(n)]
    Y = [torch.empty(R, 128, device=cuda) for _ in range(n)]
    WT = torch.empty(n, 128, 128, device=cuda)
    st = (ops.ChainStage * n)(*[ops.ChainStage(W[i].data_ptr(), B[i].data_ptr(), Z[i].data_ptr(), Y[i].data_ptr(),
                                               WT[i].data_ptr(), flags[i]) for i in range(n)])
    call("x2g_chain_fwd", ptr(x), ptr(res), st, n, R, 128, None, stream_ptr())
    dy = torch.randn(R, 128, device=cuda, generator=g)
    outs = []
    for use_wt in (True, False):
        DZ = [torch.empty(R, 128, device=cuda) for _ in range(n)]
        dx, dres = torch.empty(R, 128, device=cuda), torch.empty(R, 128, device=cuda)
        bst = (ops.ChainBwdStage * n)(*[ops.ChainBwdStage(W[i].data_ptr(), WT[i].data_ptr() if use_wt else None,
                                                          Z[i].data_ptr(), DZ[i].data_ptr(), flags[i]) for i in range(n)])
        call("x2g_chain_bwd", ptr(dy), None, bst, n, R, 128, ptr(dx), ptr(dres), None, stream_ptr())
        outs.append((dx, dres, DZ))
    torch.cuda.synchronize()
    for i in range(n):
        assert torch.equal(WT[i], W[i].t())
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    for a, b in zip(outs[0][2], outs[1][2]):
        assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("R,RR", [(21058, 6), (1000, 6), (37, 8), (5, 3)])
def test_conv_projections_fused_vs_layerwise(cuda, R, RR):
    """x2g_conv_proj_fwd / _bwd + gate backward + T-layout weight gradients (ops._ConvProjFusedFn)
    against the layer-by-layer kernels (ops._ConvProjFn) and fp64 torch: q, k, v, skip and every
    input / parameter gradient of SBFTransformerConv's projections (sbftransformer_conv.py:99-107,127)."""
    from x2gnn import ops

    g = torch.Generator(device=cuda).manual_seed(R + RR)
    x = torch.randn(R, 128, device=cuda, generator=g)
    rbf = torch.rand(R, RR, device=cuda, generator=g)
    wr = torch.randn(128, RR, device=cuda, generator=g) / 2
    W = [torch.randn(128, 128, device=cuda, generator=g) / 11.3 for _ in range(4)]
    B = [0.1 * torch.randn(128, device=cuda, generator=g) for _ in range(4)]
    gs = [torch.randn(R, 128, device=cuda, generator=g) for _ in range(4)]

    def run(fn, dtype):
        ins = [t.detach().to(dtype).requires_grad_(True) for t in [x, rbf, wr] + [v for p in zip(W, B) for v in p]]
        if fn is None:  # torch reference
            xx, rb, w_r = ins[:3]
            xs = xx * (rb @ w_r.t())
            outs = [xx @ ins[3].t() + ins[4], xs @ ins[5].t() + ins[6], xs @ ins[7].t() + ins[8],
                    xx @ ins[9].t() + ins[10]]
        else:
            outs = fn.apply(*ins)
        torch.autograd.backward(outs, [t.to(dtype) for t in gs])
        return [o.detach() for o in outs], [t.grad for t in ins]

    o_f, g_f = run(ops._ConvProjFusedFn, torch.float32)
    o_l, g_l = run(ops._ConvProjFn, torch.float32)
    o_r, g_r = run(None, torch.float64)
    for a, b, r in zip(o_f, o_l, o_r):
        torch.testing.assert_close(a.double(), r, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5)
    for i, (a, b, r) in enumerate(zip(g_f, g_l, g_r)):
        scale = float(r.abs().max()) + 1e-30
        assert float((a.double() - r).abs().max()) <= 2e-5 * scale + 1e-6, i
        assert float((a - b).abs().max()) <= 2e-5 * scale + 1e-6, i


TABLE_TREES = {
    # X2-GNN's: embedding Linear (SiLU) -> edgenn (Linear, SiLU, Linear) -> four lin_edge (no bias)
    "x2gnn": ([(-1, 1, True), (0, 1, True), (1, 0, True), (2, 0, False), (2, 0, False), (2, 0, False),
               (2, 0, False)], (3, 4, 5, 6)),
    # leaves at several depths (one a child of the input), an inner stage with its own output gradient
    "mixed": ([(-1, 1, True), (0, 0, True), (-1, 0, False), (1, 1, True), (0, 0, False)], (1, 2, 3, 4)),
    # a plain chain: one leaf, one workgroup each way
    "chain": ([(-1, 1, True), (0, 1, True), (1, 0, False)], (2,)),
}


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 10, 16])
@pytest.mark.parametrize("tree", sorted(TABLE_TREES))
def test_table_chain_vs_torch(cuda, R, tree):
    """x2g_table_chain_fwd / _bwd_ex (ops.table_chain): a tree of Linear stages on the element table
    (one workgroup per root-to-leaf path forward; the leaf stages side by side, then the inner ones,
    backward) — outputs and every input / parameter gradient vs fp64 torch, only some outputs
    receiving a gradient (as in the trunk); plus the bucket-accumulating path (grad_sink) against the
    returned gradients."""
    from x2gnn import ops
    from x2gnn.layers import Linear

    torch.manual_seed(R)
    spec, graded = TABLE_TREES[tree]
    lins = [Linear(128, 128, bias=hb).to(cuda) for _, _, hb in spec]
    x = (0.5 * torch.randn(R, 128, device=cuda)).requires_grad_(True)
    gys = {s: torch.randn(R, 128, device=cuda) for s in graded}
    outs = ops.table_chain(x, [(m, a, p) for m, (p, a, _) in zip(lins, spec)])
    torch.autograd.backward([outs[s] for s in gys], [gys[s] for s in gys])

    xr = x.detach().double().requires_grad_(True)
    ws = [m.weight.detach().double().requires_grad_(True) for m in lins]
    bs = [m.bias.detach().double().requires_grad_(True) if m.bias is not None else None for m in lins]
    ys = []
    for s, (p, a, _) in enumerate(spec):
        z = (xr if p < 0 else ys[p]) @ ws[s].t() + (bs[s] if bs[s] is not None else 0)
        ys.append(torch.nn.functional.silu(z) if a else z)
    torch.autograd.backward([ys[s] for s in gys], [gys[s].double() for s in gys])
    for a, r in zip(outs, ys):
        torch.testing.assert_close(a.detach().double(), r.detach(), rtol=1e-5, atol=1e-5)
    pairs = [(x.grad, xr.grad)] + [(m.weight.grad, w.grad) for m, w in zip(lins, ws)]
    pairs += [(m.bias.grad, b.grad) for m, b in zip(lins, bs) if b is not None]
    for i, (a, r) in enumerate(pairs):
        scale = float(r.abs().max()) + 1e-30
        assert float((a.double() - r).abs().max()) <= 2e-5 * scale + 1e-6, i

    # bucket-backed parameters: the kernel adds into the existing .grad buffers
    ref = [(m.weight.grad.clone(), m.bias.grad.clone() if m.bias is not None else None) for m in lins]
    for m in lins:
        for p in m.parameters():
            p._x2g_grad_sink = True
    outs = ops.table_chain(x.detach(), [(m, a, p) for m, (p, a, _) in zip(lins, spec)])
    torch.autograd.backward([outs[s] for s in gys], [gys[s] for s in gys])
    for m, (gw, gb) in zip(lins, ref):
        torch.testing.assert_close(m.weight.grad, 2 * gw, rtol=1e-6, atol=1e-7)
        if gb is not None:
            torch.testing.assert_close(m.bias.grad, 2 * gb, rtol=1e-6, atol=1e-7)


@pytest.mark.gpu
@pytest.mark.parametrize("R", [1, 37, 1000])
def test_featurize_vs_torch(cuda, R):
    """x2g_feat_fwd / x2g_feat_bwd + the strided T-layout weight gradients (ops.featurize) vs fp64
    torch: neo_x = SiLU(emb_trans(SiLU(mat_trans(edge_attr * env)))) (xgnn.py:64-67), 338 -> 256 ->
    128; partial 32-row tiles and an odd row count (the staged span ends mid-float4); then the
    gradient-bucket path with deferred slab sums against the returned gradients."""
    from x2gnn import ops
    from x2gnn.layers import Linear

    torch.manual_seed(R)
    x = 0.3 * torch.randn(R, 338, device=cuda)
    env = torch.rand(R, device=cuda) + 0.5
    l1, l2 = Linear(338, 256).to(cuda), Linear(256, 128).to(cuda)
    assert ops.featurize_supported(x, env, l1, l2)
    gy = torch.randn(R, 128, device=cuda)
    y = ops.featurize(x, env, l1, l2)
    y.backward(gy)

    ps = [p.detach().double().requires_grad_(True) for p in (l1.weight, l1.bias, l2.weight, l2.bias)]
    h = torch.nn.functional.silu((x.double() * env.double()[:, None]) @ ps[0].t() + ps[1])
    yr = torch.nn.functional.silu(h @ ps[2].t() + ps[3])
    yr.backward(gy.double())
    torch.testing.assert_close(y.double(), yr.detach(), rtol=1e-5, atol=1e-5)
    for i, (p, r) in enumerate(zip((l1.weight, l1.bias, l2.weight, l2.bias), ps)):
        scale = float(r.grad.abs().max()) + 1e-30
        assert float((p.grad.double() - r.grad).abs().max()) <= 2e-5 * scale + 1e-6, i

    ref = [p.grad.clone() for p in (l1.weight, l1.bias, l2.weight, l2.bias)]
    for p in (l1.weight, l1.bias, l2.weight, l2.bias):
        p._x2g_grad_sink = True
    with ops.deferred_wgrad():  # (the one flat T-layout launch: its own row split, equal to rounding)
        ops.featurize(x, env, l1, l2).backward(gy)
    for p, r in zip((l1.weight, l1.bias, l2.weight, l2.bias), ref):
        torch.testing.assert_close(p.grad, 2 * r, rtol=1e-5, atol=1e-6 * float(r.abs().max()))


def _t_layout(x):
    """Row-major [R, 128k] -> the tiled-transposed layout (x2g.h): 128-feature planes of 16-row
    tiles, feature-major inside a tile, padding rows zero."""
    R, F = x.shape
    nt = (R + 15) // 16
    xp = torch.zeros(nt * 16, F, device=x.device, dtype=x.dtype)
    xp[:R] = x
    planes = xp.view(nt, 16, F // 128, 128).permute(2, 0, 3, 1)  # plane, tile, feature, row
    return planes.contiguous().view(F // 128, -1)


@pytest.mark.gpu
@pytest.mark.parametrize("accum", [0, 1])
def test_slab_sum_batch_vs_torch(cuda, accum):
    """x2g_slab_sum_batch over mixed entries: few splits (256-element blocks, 4 waves of slabs) and
    many (the gate / radial partials: 64-element blocks, 16 split phases), a strided (ld, cols)
    destination, bias slabs, an element count that is not a multiple of 4 and a misaligned slab
    base (both scalar-path), more jobs than one launch takes."""
    from x2gnn import _lib, ops
    from x2gnn._lib import stream_ptr

    lib = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(11 + accum)
    specs = [(5376, 42, 256), (768, 0, 256), (16384, 128, 9), (128 * 128, 0, 40), (1030, 7, 64), (512, 0, 33),
             (300, 0, 1), (1000, 10, 32)] * 9  # 72 jobs > 60 per launch
    keep, jobs, refs = [], [], []
    for j, (nw, nb, splits) in enumerate(specs):
        pw_all = torch.randn(splits * nw + 1, device=cuda, generator=g)
        pw = pw_all[1:] if j % 8 == 5 else pw_all[:-1]  # entry 5: base 4 bytes off 16
        pb = torch.randn(splits, nb, device=cuda, generator=g) if nb else None
        strided = j % 8 == 3
        if strided:
            dw_store = torch.full((128, 300), 2.0, device=cuda)
            dst_w = dw_store[:, 40:140]
        else:
            dw_store = torch.full((nw,), 2.0, device=cuda)
            dst_w = dw_store
        db = torch.full((nb,), 3.0, device=cuda) if nb else None
        keep += [pw_all, pb, dw_store, db]
        sw = pw.view(splits, nw).double().sum(0)
        if strided:
            sw = sw.view(128, 128)[:, :100]
        refs.append((dst_w, sw + (2.0 if accum else 0.0), db,
                     pb.double().sum(0) + (3.0 if accum else 0.0) if nb else None))
        jobs.append(ops.SlabJob(pw.data_ptr(), pb.data_ptr() if nb else None,
                                dw_store.data_ptr() + (4 * 40 if strided else 0), db.data_ptr() if nb else None,
                                nw, nb, splits, 300 if strided else 0, 100 if strided else 0))
    arr = (ops.SlabJob * len(jobs))(*jobs)
    assert lib.x2g_slab_sum_batch(arr, len(jobs), accum, stream_ptr()) == 0
    torch.cuda.synchronize()
    for dst_w, rw, db, rb in refs:
        assert torch.allclose(dst_w.double(), rw, rtol=1e-5, atol=1e-4)
        if db is not None:
            assert torch.allclose(db.double(), rb, rtol=1e-5, atol=1e-4)
    for j in range(3, len(specs), 8):  # the strided destinations' other columns untouched
        store = keep[4 * j + 2]
        assert torch.equal(store[:, :40], torch.full_like(store[:, :40], 2.0))
        assert torch.equal(store[:, 140:], torch.full_like(store[:, 140:], 2.0))


@pytest.mark.gpu
@pytest.mark.parametrize("R,njobs", [(37, 3), (1000, 11), (21058, 52)])
def test_tiled_wgrad_flat_vs_torch(cuda, R, njobs):
    """x2g_tiled_wgrad_flat: every job's dW = dy^T x and db = colsum(dy) from T-layout operands,
    jobs concatenated over two workgroups per CU (a workgroup may span two jobs), partials summed by
    the returned slab jobs; strided (ld, cols) destinations and bias-less jobs included."""
    import ctypes
    from x2gnn import _lib, ops
    from x2gnn._lib import ptr, stream_ptr

    lib = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(R + njobs)
    dys = [torch.randn(R, 128, device=cuda, generator=g) for _ in range(njobs)]
    xs = [torch.randn(R, 128, device=cuda, generator=g) for _ in range(njobs)]
    dy_t = [_t_layout(t)[0].contiguous() for t in dys]
    x_t = [_t_layout(t)[0].contiguous() for t in xs]
    big = torch.full((128, 300), 7.0, device=cuda)  # job 1 lands as a [128, 100] block at column 50
    dws = [torch.full((128, 128), 3.0, device=cuda) for _ in range(njobs)]
    dbs = [torch.full((128,), 5.0, device=cuda) if j % 3 and j != 1 else None for j in range(njobs)]
    jobs = []
    for j in range(njobs):
        if j == 1:
            jobs.append(ops.TiledJob(dy_t[j].data_ptr(), x_t[j].data_ptr(), big.data_ptr() + 4 * 50, None, 300, 100))
        else:
            jobs.append(ops.TiledJob(dy_t[j].data_ptr(), x_t[j].data_ptr(), dws[j].data_ptr(),
                                     dbs[j].data_ptr() if dbs[j] is not None else None, 0, 0))
    arr = (ops.TiledJob * njobs)(*jobs)
    ws_bytes = int(lib.x2g_tiled_wgrad_flat_workspace(R, 128, njobs))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=cuda)
    out = (ops.SlabJob * njobs)()
    assert lib.x2g_tiled_wgrad_flat(arr, njobs, R, 128, ops.ACCUM_WGRAD | ops.DEFER_SLAB_SUM, out, ptr(ws), ws_bytes,
                                    stream_ptr()) == 0
    assert lib.x2g_slab_sum_batch(out, njobs, 1, stream_ptr()) == 0
    torch.cuda.synchronize()
    for j in range(njobs):
        ref = dys[j].double().t() @ xs[j].double()
        if j == 1:
            got = big[:, 50:150].double() - 7.0
            assert torch.equal(big[:, :50], torch.full_like(big[:, :50], 7.0))
            assert torch.equal(big[:, 150:], torch.full_like(big[:, 150:], 7.0))
            ref = ref[:, :100]
        else:
            got = dws[j].double() - 3.0
        assert float((got - ref).abs().max()) <= 2e-5 * float(ref.abs().max()), j
        if dbs[j] is not None:
            rb = dys[j].double().sum(0)
            assert float((dbs[j].double() - 5.0 - rb).abs().max()) <= 2e-5 * float(rb.abs().max()) + 1e-4, j


@pytest.mark.gpu
@pytest.mark.parametrize("rows", [[21058] * 52 + [2304] * 10, [37, 1000, 5, 2304], [16, 1], [1000, 1000, 1000]])
def test_tiled_wgrad_flat_rows_mixed(cuda, rows):
    """x2g_tiled_wgrad_flat_rows: jobs with their own row counts in one launch (the trunk's line-node
    rows and the readout MLPs' atom rows, ops._flush_tiled) — every dW / db against fp64 torch, and with
    equal row counts bit for bit the single-row-count entry x2g_tiled_wgrad_flat."""
    import ctypes
    from x2gnn import _lib, ops
    from x2gnn._lib import ptr, stream_ptr

    lib = _lib.load()
    n = len(rows)
    g = torch.Generator(device=cuda).manual_seed(sum(rows) + n)
    dys = [torch.randn(R, 128, device=cuda, generator=g) for R in rows]
    xs = [torch.randn(R, 128, device=cuda, generator=g) for R in rows]
    dy_t = [_t_layout(t)[0].contiguous() for t in dys]
    x_t = [_t_layout(t)[0].contiguous() for t in xs]

    def run(entry_rows):
        dws = [torch.zeros(128, 128, device=cuda) for _ in range(n)]
        dbs = [torch.zeros(128, device=cuda) if j % 2 == 0 else None for j in range(n)]
        arr = (ops.TiledJob * n)(*[ops.TiledJob(dy_t[j].data_ptr(), x_t[j].data_ptr(), dws[j].data_ptr(),
                                                dbs[j].data_ptr() if dbs[j] is not None else None, 0, 0)
                                   for j in range(n)])
        out = (ops.SlabJob * n)()
        if entry_rows is None:
            r = (ctypes.c_int64 * n)(*rows)
            wsb = int(lib.x2g_tiled_wgrad_flat_rows_workspace(r, n, 128))
            ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
            assert lib.x2g_tiled_wgrad_flat_rows(arr, r, n, 128, ops.ACCUM_WGRAD | ops.DEFER_SLAB_SUM, out, ptr(ws),
                                                 wsb, stream_ptr()) == 0
        else:
            wsb = int(lib.x2g_tiled_wgrad_flat_workspace(entry_rows, 128, n))
            ws = torch.empty(wsb, dtype=torch.uint8, device=cuda)
            assert lib.x2g_tiled_wgrad_flat(arr, n, entry_rows, 128, ops.ACCUM_WGRAD | ops.DEFER_SLAB_SUM, out,
                                            ptr(ws), wsb, stream_ptr()) == 0
        assert lib.x2g_slab_sum_batch(out, n, 1, stream_ptr()) == 0
        torch.cuda.synchronize()
        return dws, dbs

    dws, dbs = run(None)
    for j in range(n):
        ref = dys[j].double().t() @ xs[j].double()
        assert float((dws[j].double() - ref).abs().max()) <= 2e-5 * float(ref.abs().max()), j
        if dbs[j] is not None:
            rb = dys[j].double().sum(0)
            assert float((dbs[j].double() - rb).abs().max()) <= 2e-5 * float(rb.abs().max()) + 1e-4, j
    if len(set(rows)) == 1:
        dws1, dbs1 = run(rows[0])
        assert all(torch.equal(a, b) for a, b in zip(dws, dws1))
        assert all((a is None and b is None) or torch.equal(a, b) for a, b in zip(dbs, dbs1))


@pytest.mark.parametrize("n,beta", [(1, 1.0), (128, 1.0), (1000, 0.5), (3, 2.0)])
def test_smooth_l1_mean_vs_torch(cuda, n, beta):
    """ops.smooth_l1_loss (x2g_smooth_l1_mean_fwd / _bwd, trainer.py:41) vs F.smooth_l1_loss:
    both branches (|d| < beta and beyond), mean reduction, a non-unit upstream gradient."""
    from x2gnn import ops

    g = torch.Generator(device=cuda).manual_seed(n)
    pred = (3 * torch.randn(n, device=cuda, generator=g)).requires_grad_(True)
    target = torch.randn(n, device=cuda, generator=g)
    ref_pred = pred.detach().clone().requires_grad_(True)
    loss = ops.smooth_l1_loss(pred, target, beta=beta)
    ref = torch.nn.functional.smooth_l1_loss(ref_pred, target, beta=beta)
    assert loss.grad_fn is not None and "SmoothL1Mean" in type(loss.grad_fn).__name__
    torch.testing.assert_close(loss, ref, rtol=1e-6, atol=1e-7)
    up = torch.tensor(0.37, device=cuda)
    loss.backward(up)
    ref.backward(up)
    torch.testing.assert_close(pred.grad, ref_pred.grad, rtol=1e-6, atol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 128, 1000])
def test_smooth_l1_unit_seed_gradient_equals_backward_kernel(cuda, n):
    """ops.smooth_l1_loss(unit_seed=s): the forward launch writes d loss / d pred for the seed s (== 1) and
    the backward handed s returns it without a launch — bitwise the backward kernel's gradient for a
    ones seed; any other seed object still takes the kernel (the Trainer's step, train.py)."""
    from x2gnn import ops

    g = torch.Generator(device=cuda).manual_seed(n + 1)
    base = 3 * torch.randn(n, device=cuda, generator=g)
    target = torch.randn(n, device=cuda, generator=g)
    seed = torch.ones((), device=cuda)
    p1, p2, p3 = (base.clone().requires_grad_(True) for _ in range(3))
    l1 = ops.smooth_l1_loss(p1, target, unit_seed=seed)
    l2 = ops.smooth_l1_loss(p2, target)
    assert torch.equal(l1, l2)
    torch.autograd.backward(l1, seed)
    torch.autograd.backward(l2, torch.ones((), device=cuda))
    assert torch.equal(p1.grad, p2.grad)
    l3 = ops.smooth_l1_loss(p3, target, unit_seed=seed)
    torch.autograd.backward(l3, torch.full((), 0.5, device=cuda))  # not the seed object: the kernel
    torch.testing.assert_close(p3.grad, 0.5 * p2.grad, rtol=0, atol=0)


# ------------------------------------------------------------------------------ center-atom attention
def _sym_lg(ei, n, cuda, with_transpose=False):
    """Symmetric line graph with the center-atom outputs (edge_rev, rev_trip), its src_type / dst_type
    element rows from random atom elements, and its max degree."""
    from x2gnn import ops

    e = torch.from_numpy(ei.astype(np.int64)).to(cuda)
    T = int(triplets.vertex_to_edge(ei, n)[0].shape[1])
    ei32 = ops._i32(e)
    lg = ops.LineGraph(ei32[0].contiguous(), ei32[1].contiguous(), n, T, symmetric=True,
                       with_transpose=with_transpose)
    z = torch.randint(0, 10, (n,), generator=torch.Generator().manual_seed(n)).to(cuda)
    lg.dst_type = ops._i32(z[e[1]])
    lg.src_type = ops._i32(z[e[0]])
    deg = np.bincount(ei[0], minlength=n)
    lg.max_degree = int(deg.max()) if ei.shape[1] else 0
    lg.center_order = torch.from_numpy(np.argsort(-deg, kind="stable").astype(np.int32)).to(cuda)
    # the workgroup packs the model's batches carry (data.center_packs): (order, pack_ptr, max rows)
    from x2gnn.data import center_packs

    po, pp, pr = center_packs(deg)
    lg.packed = (torch.from_numpy(po).to(cuda), torch.from_numpy(pp).to(cuda), pr)
    return lg


def _pack_info(lg, order):
    """The fused forward's atom_info for the atoms in ``order``: (atom, first out-edge, degree, element row of
    its out-edges) per position, int32 [N * 4], from the line graph's own arrays (as collate makes it)."""
    o = order.long()
    rp = lg.atom_rowptr.long()
    first, deg = rp[o], rp[o + 1] - rp[o]
    er = lg.src_type.long()[first.clamp(max=max(lg.E - 1, 0))] if lg.E else torch.zeros_like(first)
    return torch.stack([o, first, deg, torch.where(deg > 0, er, 0)], 1).to(torch.int32).contiguous().reshape(-1)


def _attn_inputs(lg, cuda, seed, rows=10):
    g = torch.Generator(device=cuda).manual_seed(seed)
    E, T = lg.E, lg.T
    q, k, v, skip = (torch.randn(E, 128, device=cuda, generator=g) for _ in range(4))
    S = torch.randn(T, 128, device=cuda, generator=g)
    table = torch.randn(rows, 128, device=cuda, generator=g)
    return q, k, v, skip, S, table


def _fwd_both(lg, q, k, v, skip, S, table, mode, heads, channels, stats=True, order=None):
    """(center outputs, destination-major outputs): out, alpha, smax, sden, row_stats; ``order``: the center
    kernel's workgroup -> atom order (None: identity)."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr

    E, T, H, D = lg.E, lg.T, heads, heads * channels
    res = []
    for center in (True, False):
        out = torch.full((E, D), float("nan"), device=q.device)
        alpha = torch.full((T, H), float("nan"), device=q.device)
        smax, sden = torch.empty(E, H, device=q.device), torch.empty(E, H, device=q.device)
        rs = torch.empty(E, 2, device=q.device) if stats else None
        edge = table if mode == ops.EDGE_PER_DST else None
        if center:
            call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(edge),
                 ptr(lg.src_type) if edge is not None else None, mode, ptr(S), 0, ptr(lg.atom_rowptr),
                 ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(order), 0, lg.N, lg.max_degree, E, T, heads, channels, ptr(out),
                 ptr(alpha), ptr(smax), ptr(sden), ptr(rs), stream_ptr())
        else:
            call("x2g_sbf_attention_fwd_stats" if stats else "x2g_sbf_attention_fwd", ptr(q), ptr(k), ptr(v),
                 ptr(skip), ptr(edge), ptr(lg.dst_type) if edge is not None else None, mode, ptr(S), None, None,
                 ptr(lg.trip_rowptr), ptr(lg.trip_src), E, T, heads, channels, D, ptr(out), ptr(alpha), ptr(smax),
                 ptr(sden), *((ptr(rs),) if stats else ()), stream_ptr())
        res.append((out, alpha, smax, sden, rs))
    return res


def _close_fwd(a, b, tol=2e-6):
    out, alpha, smax, sden, rs = a
    out2, alpha2, smax2, sden2, rs2 = b
    assert not torch.isnan(out).any() and not torch.isnan(alpha).any()
    for x, y in ((out, out2), (alpha, alpha2), (smax, smax2)):
        torch.testing.assert_close(x, y, rtol=tol, atol=tol)
    torch.testing.assert_close(sden, sden2, rtol=1e-5, atol=1e-6)
    if rs is not None:
        torch.testing.assert_close(rs, rs2, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("heads,channels", [(16, 8), (8, 16), (32, 4)])
def test_center_forward_equals_destination_major(cuda, heads, channels):
    """x2g_sbf_attention_fwd_center (one workgroup per center atom, k / v staged in LDS) == the
    destination-major forward on a config-2 batch (128 S160 molecules), with the element-table edge term
    and without, with and without the LayerNorm row statistics; fp32 rounding apart (per-batch softmax
    rescale, 4-channel partial head sums)."""
    from x2gnn import ops
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(128, "S160", seed=11))
    lg = _sym_lg(b.edge_index.numpy(), b.num_nodes, cuda)
    assert lg.max_degree >= 9
    q, k, v, skip, S, table = _attn_inputs(lg, cuda, 3)
    for mode in (ops.EDGE_PER_DST, ops.EDGE_NONE):
        for stats in (True, False):  # (with stats: atoms launched by decreasing degree, as the model does)
            a, r = _fwd_both(lg, q, k, v, skip, S, table, mode, heads, channels, stats,
                             order=lg.center_order if stats else None)
            _close_fwd(a, r)


def test_center_forward_edge_cases(cuda):
    """Degree-1 atoms (destinations without triplets: out = skip, max -inf, denominator 0), isolated atoms
    (no edges), a hub of degree 100 (a 100 KB LDS image, above the 64 KB default), and the atom / triplet
    offsets the tiled inference path
    hands over (two molecule ranges == the whole)."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr

    # a path a-b-c (degrees 1, 2, 1), an isolated atom, a star of degree 64, a triangle
    pairs = [(0, 1), (1, 2)] + [(4, 5 + i) for i in range(100)] + [(105, 106), (106, 107), (105, 107)]
    ed = sorted({(a, b) for a, b in pairs} | {(b, a) for a, b in pairs})
    ei = np.array(ed, dtype=np.int64).T
    n = 108
    lg = _sym_lg(ei, n, cuda)
    assert lg.max_degree == 100
    q, k, v, skip, S, table = _attn_inputs(lg, cuda, 4)
    a, r = _fwd_both(lg, q, k, v, skip, S, table, ops.EDGE_PER_DST, 16, 8)
    _close_fwd(a, r)
    d_leaf = int(np.nonzero((ei[0] == 0) & (ei[1] == 1))[0][0])  # (0 -> 1): center 1 has degree 2
    assert a[2][d_leaf].isfinite().all()
    d_hub_in = int(np.nonzero((ei[0] == 1) & (ei[1] == 0))[0][0])  # (1 -> 0): center 0 has degree 1
    torch.testing.assert_close(a[0][d_hub_in], skip[d_hub_in])
    assert bool((a[2][d_hub_in] == -float("inf")).all()) and float(a[3][d_hub_in].abs().max()) == 0.0
    # two atom ranges with S handed over from each range's first triplet (the tiled path)
    split = 4  # atoms 0..3 | 4..107: the ranges' triplets are disjoint and contiguous
    t_split = int(lg.trip_rowptr[int(lg.atom_rowptr[split])])
    out = torch.empty_like(q)
    alpha = torch.empty(lg.T, 16, device=cuda)
    smax, sden, rs = torch.empty(lg.E, 16, device=cuda), torch.empty(lg.E, 16, device=cuda), torch.empty(lg.E, 2, device=cuda)
    for a0, a1, t0, t1 in ((0, split, 0, t_split), (split, n, t_split, lg.T)):
        Sc = S[t0:t1].clone()
        call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
             ops.EDGE_PER_DST, ptr(Sc), t0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), None, a0, a1 - a0,
             lg.max_degree, lg.E, lg.T, 16, 8, ptr(out), ptr(alpha), ptr(smax), ptr(sden), ptr(rs), stream_ptr())
    for x, y in zip((out, alpha, smax, sden, rs), a):
        assert torch.equal(x, y)


def _bwd_both(lg, q, k, v, S, table, mode, heads, channels, seed):
    """(center, destination-major fold) backward outputs on the same forward state: dq, dk, dv, G and the
    element-table gradient of the edge term (keyed sums in fp64), then the center kernel's per-atom
    edge-term rows raw."""
    from x2gnn import _lib, ops
    from x2gnn._lib import call, ptr, stream_ptr

    E, T, H, D = lg.E, lg.T, heads, heads * channels
    skip = torch.zeros_like(q)
    (out, alpha, smax, sden, _), _ = _fwd_both(lg, q, k, v, skip, S, table, mode, heads, channels, stats=False)
    g = torch.Generator(device=q.device).manual_seed(seed)
    dout = torch.randn(E, D, device=q.device, generator=g)
    y = torch.randn(T, 8, device=q.device, generator=g)
    y[:, 7] = 1.0
    edge = table if mode == ops.EDGE_PER_DST else None
    rows = table.shape[0]
    f = dict(device=q.device, dtype=torch.float32)
    # center
    dq, dk, dv = (torch.full((E, D), float("nan"), **f) for _ in range(3))
    G = torch.full((E, 8, D), float("nan"), **f)
    de_atom = torch.full((lg.N, D), float("nan"), **f) if edge is not None else None
    assert int(_lib.load().x2g_sbf_attention_bwd_center_lds(lg.max_degree, heads)) <= 160 * 1024
    call("x2g_sbf_attention_bwd_center", ptr(q), ptr(k), ptr(v), ptr(edge), ptr(lg.src_type) if edge is not None else None,
         mode, ptr(S), None, None, ptr(y), ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(lg.center_order),
         ptr(alpha), ptr(smax), ptr(sden), ptr(dout), lg.N, lg.max_degree, E, T, heads, channels, ptr(dq), ptr(dk),
         ptr(dv), ptr(G), ptr(de_atom), ptr(torch.empty(2, T, H, **f)), stream_ptr())
    c = [dq, dk, dv, G]
    if edge is not None:
        c.append(torch.zeros(rows, D, dtype=torch.float64, device=q.device).index_add_(0, lg.atom_type.long(), de_atom.double()))
    # destination-major fold passes
    dq2, dk2, dv2 = (torch.empty(E, D, **f) for _ in range(3))
    G2 = torch.empty(E, 8, D, **f)
    prob, rho = torch.empty(T, H, **f), torch.empty(E, H, **f)
    de = torch.empty(E, D, **f) if edge is not None else None
    call("x2g_sbf_attention_bwd_dst_g", ptr(q), ptr(k), ptr(v), ptr(edge), ptr(lg.dst_type) if edge is not None else None,
         mode, ptr(S), ptr(lg.trip_rowptr), ptr(lg.trip_src), ptr(alpha), ptr(smax), ptr(sden), ptr(dout), E, T, heads,
         channels, ptr(dq2), ptr(de), None, ptr(prob), ptr(rho), stream_ptr())
    src_rowptr, src_perm = lg.src_csr()
    call("x2g_sbf_attention_bwd_src_fold", ptr(q), ptr(v), ptr(edge), ptr(lg.dst_type) if edge is not None else None,
         ptr(lg.src_type) if edge is not None else None, rows if edge is not None else 0, mode, ptr(S), ptr(y),
         ptr(src_rowptr), ptr(src_perm), ptr(lg.src_dst), ptr(lg.trip_dst), ptr(prob), None, ptr(rho), ptr(dout), E, T,
         heads, channels, ptr(dk2), ptr(dv2), ptr(G2), stream_ptr())
    r = [dq2, dk2, dv2, G2]
    if edge is not None:
        r.append(torch.zeros(rows, D, dtype=torch.float64, device=q.device).index_add_(0, lg.dst_type.long(), de.double()))
    return c, r


def _close_bwd(c, r):
    for name, x, y in zip(("dq", "dk", "dv", "G", "d_edge"), c, r):
        assert not torch.isnan(x).any(), name
        scale = float(y.abs().max())
        err = float((x.double() - y.double()).abs().max())
        assert err <= 2e-5 * scale + 1e-6, (name, err, scale)


@pytest.mark.parametrize("heads,channels", [(16, 8), (8, 16), (32, 4)])
def test_center_backward_equals_fold_passes(cuda, heads, channels):
    """x2g_sbf_attention_bwd_center (both backward passes in one launch per center atom) == the
    destination-major x2g_sbf_attention_bwd_dst_g + source-major x2g_sbf_attention_bwd_src_fold on a
    config-2 batch: dq, dk, dv, the folded lin_sbf gradient G, and the element-table gradient (per-atom
    rows keyed by element == per-destination rows keyed by destination element), with and without the
    edge term; within 2e-5 of each output's max (fp32 reassociation)."""
    from x2gnn import ops
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(128, "S160", seed=12))
    lg = _sym_lg(b.edge_index.numpy(), b.num_nodes, cuda, with_transpose=True)
    lg.atom_type = ops._i32(torch.randint(0, 10, (b.num_nodes,), generator=torch.Generator().manual_seed(b.num_nodes)).to(cuda))
    lg.src_type = ops._i32(lg.atom_type[lg.edge_src.long()])
    lg.dst_type = ops._i32(lg.atom_type[lg.edge_dst.long()])
    q, k, v, _, S, table = _attn_inputs(lg, cuda, 5)
    for mode in (ops.EDGE_PER_DST, ops.EDGE_NONE):
        c, r = _bwd_both(lg, q, k, v, S, table, mode, heads, channels, 6)
        _close_bwd(c, r)


def test_center_backward_edge_cases(cuda):
    """Degree-1 and isolated atoms (zero rows), a hub of degree 24, a triangle; vs the fold passes.  A
    degree above X2G_CENTER_MAX_DEGREE is refused (X2G_EUNSUPPORTED: the host then takes the fold
    passes)."""
    from x2gnn import ops

    pairs = [(0, 1), (1, 2)] + [(4, 5 + i) for i in range(24)] + [(29, 30), (30, 31), (29, 31)]
    ed = sorted({(a, b) for a, b in pairs} | {(b, a) for a, b in pairs})
    ei = np.array(ed, dtype=np.int64).T
    n = 32
    lg = _sym_lg(ei, n, cuda, with_transpose=True)
    z = torch.randint(0, 10, (n,), generator=torch.Generator().manual_seed(1)).to(cuda)
    lg.atom_type = ops._i32(z)
    lg.src_type, lg.dst_type = ops._i32(z[lg.edge_src.long()]), ops._i32(z[lg.edge_dst.long()])
    q, k, v, _, S, table = _attn_inputs(lg, cuda, 7)
    c, r = _bwd_both(lg, q, k, v, S, table, ops.EDGE_PER_DST, 16, 8, 8)
    _close_bwd(c, r)
    from x2gnn import _lib

    assert int(_lib.load().x2g_sbf_attention_bwd_center_lds(130, 16)) > 160 * 1024 or 130 > ops.CENTER_MAX_DEGREE
    rc = _lib.load().x2g_sbf_attention_bwd_center(None, None, None, None, None, 0, None, None, None, None, None, None,
                                                   None, None, None, None, None, None, 1, 130, 1, 1, 16, 8, None, None,
                                                   None, None, None, None, None)
    assert rc == 1002  # X2G_EUNSUPPORTED


def test_center_forward_fused_projection_equals_projected(cuda):
    """x2g_sbf_attention_fwd_center_sf (S_t = b + sum_l Y_l(t) P_s[l] rebuilt per center atom from the sbf
    factors, no S read) == x2g_sbf_project + x2g_sbf_attention_fwd_center on a config-2 batch: outputs,
    logits, softmax statistics, row statistics, and the S rows it stores for the backward; and without the
    S store (inference) the same outputs.  fp32 reassociation of the 42-term projection: 1e-5."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(128, "S160", seed=13))
    lg = _sym_lg(b.edge_index.numpy(), b.num_nodes, cuda)
    E, T, H, C, D = lg.E, lg.T, 16, 8, 128
    g = torch.Generator(device=cuda).manual_seed(14)
    q, k, v, skip = (torch.randn(E, D, device=cuda, generator=g) for _ in range(4))
    table = torch.randn(10, D, device=cuda, generator=g)
    radial = torch.randn(E, 42, device=cuda, generator=g)
    y = torch.randn(T, 8, device=cuda, generator=g)
    y[:, 7] = 1.0
    sbf = (radial[lg.trip_src.long()].view(T, 7, 6) * y[:, :7, None]).reshape(T, 42).contiguous()
    W = 0.2 * torch.randn(D, 42, device=cuda, generator=g)
    bias = 0.1 * torch.randn(D, device=cuda, generator=g)
    f = dict(device=cuda, dtype=torch.float32)
    S = torch.empty(T, D, **f)
    call("x2g_sbf_project", ptr(sbf), T, 42, ptr(W), ptr(bias), D, ptr(S), stream_ptr())
    ref = [torch.empty(E, D, **f), torch.empty(T, H, **f), torch.empty(E, H, **f), torch.empty(E, H, **f),
           torch.empty(E, 2, **f)]
    call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
         ops.EDGE_PER_DST, ptr(S), 0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(lg.center_order), 0,
         lg.N, lg.max_degree, E, T, H, C, *[ptr(t) for t in ref], stream_ptr())
    po, pp, pr = lg.packed
    runs = []
    for store, packed in ((True, False), (False, False), (True, True), (False, True)):
        got = [torch.full_like(t, float("nan")) for t in ref]
        S2 = torch.full((T, D), float("nan"), **f) if store else None
        # unpacked: identity order with the S store, the degree order without; packed: the model's units
        order, packs, units, rows = (po, pp, int(pp.shape[0]) - 1, pr) if packed else \
            (None if store else lg.center_order, None, lg.N, lg.max_degree)
        # packed with the S store: the row ranges from atom_info (the model's launch); without: derived
        info = _pack_info(lg, po) if packed and store else None
        call("x2g_sbf_attention_fwd_center_sf", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
             ops.EDGE_PER_DST, ptr(radial), ptr(y), ptr(W), ptr(bias), ptr(lg.atom_rowptr), ptr(lg.edge_rev),
             ptr(lg.rev_trip), ptr(order), ptr(packs), ptr(info), 0, units, rows, E, T, H, C,
             *[ptr(t) for t in got], ptr(S2), None, stream_ptr())
        for name, a, r in zip(("out", "alpha", "smax", "sden", "row_stats"), got, ref):
            assert not torch.isnan(a).any(), name
            torch.testing.assert_close(a, r, rtol=1e-5, atol=1e-5, msg=name)
        if store:
            torch.testing.assert_close(S2, S, rtol=1e-5, atol=1e-5)
        runs.append(got + ([S2] if store else []))
    for a, b in zip(runs[:2], runs[2:]):  # packing changes no bit
        for x, y in zip(a, b):
            assert torch.equal(x, y)


def test_center_fused_projection_packed_edge_cases(cuda):
    """The fused-projection forward over workgroup packs on a graph with degree-1 atoms, isolated atoms (in
    a unit of their own: no rows), a hub of degree 20 (above the 16-row pack capacity: alone) and small
    atoms sharing units: == the one-atom-per-workgroup launch, bitwise, and == projection + center
    forward within fp32 reassociation."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr

    pairs = [(0, 1), (1, 2)] + [(4, 5 + i) for i in range(20)] + [(25, 26), (26, 27), (25, 27)] + \
        [(28 + i, 29 + i) for i in range(6)]
    ed = sorted({(a, b) for a, b in pairs} | {(b, a) for a, b in pairs})
    ei = np.array(ed, dtype=np.int64).T
    n = 36  # atoms 3 and 35 have no edges
    lg = _sym_lg(ei, n, cuda)
    po, pp, pr = lg.packed
    assert pr == 20 and int(pp.shape[0]) - 1 < n
    E, T, H, C, D = lg.E, lg.T, 16, 8, 128
    g = torch.Generator(device=cuda).manual_seed(15)
    q, k, v, skip = (torch.randn(E, D, device=cuda, generator=g) for _ in range(4))
    table = torch.randn(10, D, device=cuda, generator=g)
    radial = torch.randn(E, 42, device=cuda, generator=g)
    y = torch.randn(T, 8, device=cuda, generator=g)
    y[:, 7] = 1.0
    sbf = (radial[lg.trip_src.long()].view(T, 7, 6) * y[:, :7, None]).reshape(T, 42).contiguous()
    W = 0.2 * torch.randn(D, 42, device=cuda, generator=g)
    bias = 0.1 * torch.randn(D, device=cuda, generator=g)
    f = dict(device=cuda, dtype=torch.float32)
    S = torch.empty(T, D, **f)
    call("x2g_sbf_project", ptr(sbf), T, 42, ptr(W), ptr(bias), D, ptr(S), stream_ptr())
    ref = [torch.empty(E, D, **f), torch.empty(T, H, **f), torch.empty(E, H, **f), torch.empty(E, H, **f),
           torch.empty(E, 2, **f)]
    call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
         ops.EDGE_PER_DST, ptr(S), 0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), None, 0,
         lg.N, lg.max_degree, E, T, H, C, *[ptr(t) for t in ref], stream_ptr())
    runs = []
    for packed in (False, True):
        got = [torch.full_like(t, float("nan")) for t in ref]
        S2 = torch.full((T, D), float("nan"), **f)
        order, packs, units, rows = (po, pp, int(pp.shape[0]) - 1, pr) if packed else (None, None, lg.N, lg.max_degree)
        info = _pack_info(lg, po) if packed else None
        call("x2g_sbf_attention_fwd_center_sf", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
             ops.EDGE_PER_DST, ptr(radial), ptr(y), ptr(W), ptr(bias), ptr(lg.atom_rowptr), ptr(lg.edge_rev),
             ptr(lg.rev_trip), ptr(order), ptr(packs), ptr(info), 0, units, rows, E, T, H, C, *[ptr(t) for t in got], ptr(S2),
             None, stream_ptr())
        for name, a, r in zip(("out", "alpha", "smax", "sden", "row_stats"), got, ref):
            torch.testing.assert_close(a, r, rtol=1e-5, atol=1e-5, msg=name, equal_nan=False)
        torch.testing.assert_close(S2, S, rtol=1e-5, atol=1e-5)
        runs.append(got + [S2])
    for x, yy in zip(*runs):
        assert torch.equal(x, yy)


def test_center_backward_from_p_rows_equals_s_rows(cuda):
    """The fused forward's P rows (sbf_p_out [E, 7, 128]: 3.5 KB per source instead of 512 B per triplet)
    feed the center backward, which rebuilds S_t = b + sum_l Y_l(t) P_s[l] in the forward's own arithmetic:
    every backward output equals the one from the S rows the same forward stores, bit for bit, with and
    without the edge term — the P-row form given no logits (it recomputes them as the forward formed them);
    and the P rows equal W R_s per source (fp32)."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(128, "S160", seed=16))
    lg = _sym_lg(b.edge_index.numpy(), b.num_nodes, cuda)
    z = torch.randint(0, 10, (b.num_nodes,), generator=torch.Generator().manual_seed(2)).to(cuda)
    lg.atom_type = ops._i32(z)
    lg.src_type, lg.dst_type = ops._i32(z[lg.edge_src.long()]), ops._i32(z[lg.edge_dst.long()])
    E, T, H, C, D = lg.E, lg.T, 16, 8, 128
    g = torch.Generator(device=cuda).manual_seed(17)
    q, k, v, skip, dout = (torch.randn(E, D, device=cuda, generator=g) for _ in range(5))
    table = torch.randn(10, D, device=cuda, generator=g)
    radial = torch.randn(E, 42, device=cuda, generator=g)
    y = torch.randn(T, 8, device=cuda, generator=g)
    y[:, 7] = 1.0
    W = 0.2 * torch.randn(D, 42, device=cuda, generator=g)
    bias = 0.1 * torch.randn(D, device=cuda, generator=g)
    f = dict(device=cuda, dtype=torch.float32)
    po, pp, pr = lg.packed
    for mode in (ops.EDGE_PER_DST, ops.EDGE_NONE):
        edge = table if mode == ops.EDGE_PER_DST else None
        # the forward of this mode (the P-row backward recomputes this forward's logits)
        fw = [torch.empty(E, D, **f), torch.empty(T, H, **f), torch.empty(E, H, **f), torch.empty(E, H, **f),
              torch.empty(E, 2, **f)]
        S, P = torch.full((T, D), float("nan"), **f), torch.full((E, 7, D), float("nan"), **f)
        call("x2g_sbf_attention_fwd_center_sf", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(edge),
             ptr(lg.src_type) if edge is not None else None, mode, ptr(radial), ptr(y), ptr(W), ptr(bias),
             ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(po), ptr(pp), ptr(_pack_info(lg, po)), 0,
             int(pp.shape[0]) - 1, pr, E, T, H, C, *[ptr(t) for t in fw], ptr(S), ptr(P), stream_ptr())
        ref_p = torch.einsum("clk,elk->elc", W.view(D, 7, 6), radial.view(E, 7, 6))
        torch.testing.assert_close(P, ref_p, rtol=1e-5, atol=1e-5)
        alpha, smax, sden = fw[1], fw[2], fw[3]
        outs = []
        for from_p in (False, True):
            dq, dk, dv = (torch.full((E, D), float("nan"), **f) for _ in range(3))
            G = torch.full((E, 8, D), float("nan"), **f)
            de = torch.full((lg.N, D), float("nan"), **f) if edge is not None else None
            call("x2g_sbf_attention_bwd_center", ptr(q), ptr(k), ptr(v), ptr(edge),
                 ptr(lg.src_type) if edge is not None else None, mode, None if from_p else ptr(S),
                 ptr(P) if from_p else None, ptr(bias) if from_p else None, ptr(y), ptr(lg.atom_rowptr),
                 ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(lg.center_order), None if from_p else ptr(alpha), ptr(smax),
                 ptr(sden), ptr(dout), lg.N, lg.max_degree, E, T, H, C, ptr(dq), ptr(dk), ptr(dv), ptr(G), ptr(de),
                 ptr(torch.empty(2, T, H, **f)), stream_ptr())
            outs.append([t for t in (dq, dk, dv, G, de) if t is not None])
        for a, r in zip(*outs):
            assert not torch.isnan(a).any()
            assert torch.equal(a, r)


@pytest.mark.parametrize("graph", ["aid", "hub100"])
def test_center_fused_source_tiles_equal_projected(cuda, graph):
    """x2g_sbf_attention_fwd_center_sf_tiled (atoms beyond the fused forward's LDS image: sources staged 16 at
    a time, each owner's destinations carrying their online-softmax state across the tiles) == projection +
    the S-reading center forward on AID_kcal molecules (config 5's geometry: degrees up to ~50, RMAX 4) and on
    a graph with a degree-100 hub (RMAX 8), degree-1 and isolated atoms: outputs, logits, softmax and row
    statistics, the S rows and P rows it stores; the model's split launch (the leading hub units tiled, the
    packed rest untiled: data.center_hubs) gives the same outputs as all atoms tiled."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr
    from x2gnn.data import center_hubs
    from x2gnn.synth import molecules_from_geometry_file

    if graph == "aid":
        from x2gnn.data import collate

        b = collate(molecules_from_geometry_file(os.path.join(GOLDEN, "aid_geom.npz"), indices=[0, 5, 9], seed=0))
        ei, n = b.edge_index.numpy(), b.num_nodes
    else:
        pairs = [(0, 1), (1, 2)] + [(4, 5 + i) for i in range(100)] + [(110, 111), (111, 112), (110, 112)] + \
            [(5 + i, 6 + i) for i in range(30)]
        ed = sorted({(a, c) for a, c in pairs} | {(c, a) for a, c in pairs})
        ei, n = np.array(ed, dtype=np.int64).T, 114  # atoms 3 and 113 have no edges
    lg = _sym_lg(ei, n, cuda)
    deg = np.bincount(ei[0], minlength=n)
    assert lg.max_degree > 33
    E, T, H, C, D = lg.E, lg.T, 16, 8, 128
    g = torch.Generator(device=cuda).manual_seed(18)
    q, k, v, skip = (torch.randn(E, D, device=cuda, generator=g) for _ in range(4))
    table = torch.randn(10, D, device=cuda, generator=g)
    radial = torch.randn(E, 42, device=cuda, generator=g)
    y = torch.randn(T, 8, device=cuda, generator=g)
    y[:, 7] = 1.0
    sbf = (radial[lg.trip_src.long()].view(T, 7, 6) * y[:, :7, None]).reshape(T, 42).contiguous()
    W = 0.2 * torch.randn(D, 42, device=cuda, generator=g)
    bias = 0.1 * torch.randn(D, device=cuda, generator=g)
    f = dict(device=cuda, dtype=torch.float32)
    S = torch.empty(T, D, **f)
    call("x2g_sbf_project", ptr(sbf), T, 42, ptr(W), ptr(bias), D, ptr(S), stream_ptr())
    ref = [torch.empty(E, D, **f), torch.empty(T, H, **f), torch.empty(E, H, **f), torch.empty(E, H, **f),
           torch.empty(E, 2, **f)]
    call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type),
         ops.EDGE_PER_DST, ptr(S), 0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), None, 0,
         lg.N, lg.max_degree, E, T, H, C, *[ptr(t) for t in ref], stream_ptr())
    ref_p = torch.einsum("clk,elk->elc", W.view(D, 7, 6), radial.view(E, 7, 6))
    po, pp, pr = lg.packed
    hubs, rows = center_hubs(deg, po.cpu().numpy(), pp.cpu().numpy())
    assert 0 < hubs < int(pp.shape[0]) - 1 and rows <= 17
    info = _pack_info(lg, po)
    runs = []
    for split in (False, True):
        got = [torch.full_like(t, float("nan")) for t in ref]
        S2 = torch.full((T, D), float("nan"), **f)
        P2 = torch.full((E, 7, D), float("nan"), **f)
        common = (ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type), ops.EDGE_PER_DST, ptr(radial),
                  ptr(y), ptr(W), ptr(bias), ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip))
        outs = (E, T, H, C, *[ptr(t) for t in got], ptr(S2), ptr(P2), stream_ptr())
        if split:  # the model's launches
            call("x2g_sbf_attention_fwd_center_sf_tiled", *common, ptr(po), ptr(pp), ptr(info), 0, hubs,
                 lg.max_degree, 0, *outs)
            call("x2g_sbf_attention_fwd_center_sf", *common, ptr(po), ptr(pp), ptr(info), hubs,
                 int(pp.shape[0]) - 1 - hubs, rows, *outs)
        else:  # every atom tiled, by decreasing degree, row ranges derived
            call("x2g_sbf_attention_fwd_center_sf_tiled", *common, ptr(lg.center_order), None, None, 0, lg.N,
                 lg.max_degree, 0, *outs)
        for name, a, r in zip(("out", "alpha", "smax", "sden", "row_stats"), got, ref):
            assert not torch.isnan(a).any(), name
            torch.testing.assert_close(a, r, rtol=1e-5, atol=1e-5, msg=name)
        torch.testing.assert_close(S2, S, rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(P2, ref_p, rtol=1e-5, atol=1e-5)
        runs.append(got)
    for a, r in zip(*runs):  # the hubs are computed by the same kernel either way; the rest to fp32 rounding
        torch.testing.assert_close(a, r, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("graph", ["s160", "aid"])
def test_device_center_schedule(cuda, graph):
    """x2g_center_schedule (the center kernels' schedule made on the device, for batches without collate's):
    center_order is a permutation by non-increasing degree; every atom sits in exactly one unit, a unit of
    several atoms holds <= 16 rows and <= 16 atoms from one 64-atom window, the units come by non-increasing
    largest degree and the empty slots after them; atom_info
    matches the line graph; and the fused forward over it (both forms over all unit slots, each leaving out
    the other's units) equals the forward over collate's host schedule bit for bit."""
    from x2gnn import ops
    from x2gnn._lib import call, ptr, stream_ptr
    from x2gnn.data import center_hubs, collate
    from x2gnn.synth import molecules_from_geometry_file, synthetic_molecules

    if graph == "s160":
        b = collate(synthetic_molecules(128, "S160", seed=21))
    else:  # degrees up to ~50, molecules of more than 64 atoms (windows inside and across molecules)
        b = collate(molecules_from_geometry_file(os.path.join(GOLDEN, "aid_geom.npz"), indices=[0, 5, 9, 30], seed=0))
    ei, n = b.edge_index.numpy(), b.num_nodes
    lg = _sym_lg(ei, n, cuda)
    deg = np.bincount(ei[0], minlength=n)
    i32 = dict(dtype=torch.int32, device=cuda)
    c_order, p_order, p_ptr = torch.full((n,), -1, **i32), torch.full((n,), -1, **i32), torch.full((n + 1,), -1, **i32)
    info = torch.full((4 * n,), -1, **i32)
    ws_b = int(_lib_mod().x2g_center_schedule_workspace(n))
    ws = torch.empty(ws_b, dtype=torch.uint8, device=cuda)
    call("x2g_center_schedule", ptr(lg.atom_rowptr), ptr(lg.src_type), n, ptr(c_order), ptr(p_order), ptr(p_ptr),
         ptr(info), ptr(ws), ws_b, stream_ptr())
    co, po, pp = c_order.cpu().numpy(), p_order.cpu().numpy(), p_ptr.cpu().numpy()
    assert np.array_equal(np.sort(co), np.arange(n)) and (np.diff(deg[co]) <= 0).all()
    assert np.array_equal(np.sort(po), np.arange(n)) and pp[0] == 0 and pp[n] == n and (np.diff(pp) >= 0).all()
    keys, n_units = [], 0
    for u in range(n):
        mem = po[pp[u]:pp[u + 1]]
        if len(mem) == 0:
            continue
        assert u == n_units, "empty unit slots only after the units"
        n_units += 1
        assert (mem // 64 == mem[0] // 64).all()
        if len(mem) > 1:
            assert deg[mem].sum() <= 16 and len(mem) <= 16
        keys.append(min(deg[mem].max(), 128))
    assert (np.diff(keys) <= 0).all() and (pp[n_units:] == n).all()
    inf = info.cpu().numpy().reshape(n, 4)
    rp = lg.atom_rowptr.cpu().numpy()
    st = lg.src_type.cpu().numpy()
    assert np.array_equal(inf[:, 0], po) and np.array_equal(inf[:, 1], rp[po]) and np.array_equal(inf[:, 2], deg[po])
    assert np.array_equal(inf[:, 3], np.where(deg[po] > 0, st[np.minimum(rp[po], len(st) - 1)], 0))
    # the fused forward over the device schedule == over the host schedule
    E, T, H, C, D = lg.E, lg.T, 16, 8, 128
    g = torch.Generator(device=cuda).manual_seed(22)
    q, k, v, skip = (torch.randn(E, D, device=cuda, generator=g) for _ in range(4))
    table = torch.randn(10, D, device=cuda, generator=g)
    radial = torch.randn(E, 42, device=cuda, generator=g)
    y = torch.randn(T, 8, device=cuda, generator=g)
    y[:, 7] = 1.0
    W = 0.2 * torch.randn(D, 42, device=cuda, generator=g)
    bias = 0.1 * torch.randn(D, device=cuda, generator=g)
    f = dict(device=cuda, dtype=torch.float32)
    hpo, hpp, _ = lg.packed
    hubs, rows = center_hubs(deg, hpo.cpu().numpy(), hpp.cpu().numpy())
    runs = []
    for device_sched in (False, True):
        got = [torch.full((E, D), float("nan"), **f), torch.full((T, H), float("nan"), **f),
               torch.full((E, H), float("nan"), **f), torch.full((E, H), float("nan"), **f),
               torch.full((E, 2), float("nan"), **f), torch.full((E, 7, D), float("nan"), **f)]
        lg.pack_order, lg.center_packs = (p_order, p_ptr) if device_sched else (hpo, hpp)
        lg.pack_info = info if device_sched else _pack_info(lg, hpo)
        lg.center_rows = 17 if device_sched else rows
        lg.center_hubs, lg.center_mixed = (0, True) if device_sched else (hubs, False)
        order, packs, inf_t, launches = ops._center_split(lg)
        common = (ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(lg.src_type), ops.EDGE_PER_DST, ptr(radial),
                  ptr(y), ptr(W), ptr(bias), ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(order),
                  ptr(packs), ptr(inf_t))
        ops._center_launch(launches, common, (E, T, H, C, *[ptr(t) for t in got[:5]], None, ptr(got[5]),
                                              stream_ptr()))
        for t in got:
            assert not torch.isnan(t).any()
        runs.append(got)
    for a, r in zip(*runs):
        assert torch.equal(a, r)


def _lib_mod():
    from x2gnn import _lib

    return _lib.load()
