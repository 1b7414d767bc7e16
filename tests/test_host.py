"""Host-side logic: synthetic data, collate, module trees, generated basis constants."""
import math

import numpy as np
import pytest
import torch

from conftest import golden
from helpers import model_cfg


def test_synthetic_shapes_match_survey():
    from x2gnn.synth import synthetic_molecules

    ms = synthetic_molecules(32, "S160", seed=0)
    assert np.mean([len(m["x"]) for m in ms]) == 18
    assert 140 < np.mean([m["edge_num"] for m in ms]) < 185       # ~160 directed edges
    assert 1200 < np.mean([m["triplet_num"] for m in ms]) < 1750  # ~1460 triplets
    m = ms[0]
    ei = m["edge_index"]
    key = ei[0] * 100 + ei[1]
    assert np.all(np.diff(key) > 0)  # sorted by (src, dst), no duplicates
    assert m["edge_attr"].shape == (ei.shape[1], 338) and m["edge_attr"].dtype == np.float32


def test_synthetic_is_deterministic():
    from x2gnn.synth import synthetic_molecules

    a = synthetic_molecules(3, "S5A", seed=5)
    b = synthetic_molecules(3, "S5A", seed=5)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x["atom_pos"], y["atom_pos"])
        np.testing.assert_array_equal(x["edge_attr"], y["edge_attr"])


def test_collate_pyg_semantics():
    from x2gnn.data import collate
    from x2gnn.synth import synthetic_molecules

    ms = synthetic_molecules(3, "S160", seed=1)
    b = collate(ms)
    n = [len(m["x"]) for m in ms]
    e = [m["edge_num"] for m in ms]
    assert b.num_graphs == 3
    assert "batch" in b._store
    assert b.edge_index.shape == (2, sum(e))
    # edge_index incremented by the running atom count (PyG __inc__ for edge_index)
    np.testing.assert_array_equal(b.edge_index[:, e[0]:e[0] + e[1]].numpy(), ms[1]["edge_index"] + n[0])
    np.testing.assert_array_equal(b.edge_num.numpy(), e)
    np.testing.assert_array_equal(b.ptr.numpy(), np.concatenate([[0], np.cumsum(n)]))
    np.testing.assert_array_equal(b.batch.numpy(), np.repeat(np.arange(3), n))
    assert list(b._meta["triplets"]) == [m["triplet_num"] for m in ms]
    # reference quirk (xgnn.py:42-43): setting num_graphs on a batch must not change it
    b.num_graphs = 1
    assert b.num_graphs == 3


def test_meta_fallback_matches_collate():
    from x2gnn.data import _meta_from_tensors, collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(4, "S160", seed=2))
    m = _meta_from_tensors(b)
    for k in ("nodes", "edges", "triplets"):
        np.testing.assert_array_equal(m[k], b._meta[k])


@pytest.mark.parametrize("fixture", ["model_small.npz", "model_full.npz", "model_global.npz"])
def test_state_dict_names_equal_reference(fixture):
    import x2gnn

    z = golden(fixture)
    cls = x2gnn.xgnn_poly if str(z["kind"]) == "poly" else x2gnn.xgnn_poly_global
    m = cls(**model_cfg(z))
    assert [n for n, _ in m.named_parameters()] == list(z["param_names"])
    assert [str(tuple(p.shape)) for _, p in m.named_parameters()] == list(z["param_shapes"])
    assert list(m.state_dict().keys()) == list(z["state_keys"])


def test_generated_basis_constants_vs_oracle():
    """The device's expanded Rayleigh coefficients reproduce N_ln j_l(z_ln x) (fp64 check)."""
    from x2gnn import basis_consts as bc

    from oracle import ref_cpu

    nrad = bc.NUM_RADIAL  # 16: compiled maximum (F_B_2D(7, 16) is the reference's default)
    np.testing.assert_allclose(np.array(bc.ZEROS), ref_cpu._basis_consts(7, nrad)[0], rtol=0, atol=0)
    # the config.json basis (7 x 6) uses the first 6 columns: the same float32 zeros
    np.testing.assert_allclose(np.array(bc.ZEROS)[:, :6], ref_cpu._basis_consts(7, 6)[0], rtol=0, atol=0)
    x = np.linspace(0.15, 1.0, 61)
    ref = ref_cpu.bessel_radial(x, 7, nrad)
    coef = np.array(bc.COEF)
    for l in range(7):
        for n in range(nrad):
            z = bc.ZEROS[l][n]
            acc = np.zeros_like(x)
            for m in range(l, -1, -1):
                trig = np.sin(z * x) if m % 2 == 0 else np.cos(z * x)
                acc += coef[l, n, m] * x ** m * trig
            # the expanded Rayleigh form cancels at small z x (worst at l = 6, n = 0): fp64 here
            np.testing.assert_allclose(acc / x ** (l + 1), ref[:, nrad * l + n], rtol=1e-6, atol=1e-8)
    y = np.array(bc.YCOEF)
    c = np.cos(np.linspace(0, math.pi, 17))
    for l in range(7):
        val = sum(y[l, p] * c ** p for p in range(7))
        np.testing.assert_allclose(val, ref_cpu.sph_y0(np.arccos(c))[:, l], atol=1e-12)


def test_device_ops_refuse_cpu_tensors():
    from x2gnn import ops

    x = torch.zeros(4, 128)
    with pytest.raises(RuntimeError, match="GPU"):
        ops.segment_sum(x, torch.zeros(3, dtype=torch.int32), 2)
    with pytest.raises(RuntimeError, match="GPU"):
        ops.vertex_to_edge(torch.zeros(2, 3, dtype=torch.int64), 3, 0)


def test_center_packs_and_atom_info():
    """data.center_packs (the fused forward's workgroup units): every atom in exactly one unit, no unit
    above 16 rows unless it is one atom of larger degree, atoms without edges in units of their own, the
    units in decreasing order of their largest degree, 90 % of the owners busy at config 2; and
    collate's atom_info rows = (atom, first out-edge, degree, element) in the same order."""
    import numpy as np

    from x2gnn.data import center_packs, collate
    from x2gnn.synth import synthetic_molecules

    b = collate(synthetic_molecules(128, "S160", seed=1000))
    n = b.num_nodes
    deg = np.bincount(b.edge_index[0].numpy(), minlength=n)
    order, packs, rows = center_packs(deg)
    assert sorted(order.tolist()) == list(range(n))
    units = [order[packs[u]:packs[u + 1]] for u in range(len(packs) - 1)]
    sums = np.array([deg[u].sum() for u in units])
    assert all(s <= 16 or len(u) == 1 for s, u in zip(sums, units))
    assert rows == sums.max() and all(len(u) <= 16 for u in units)
    big = np.array([deg[u].max() for u in units])
    assert (np.diff(big) <= 0).all()
    assert sums.sum() / (16 * np.ceil(sums / 16)).sum() > 0.88
    st = b._store
    assert np.array_equal(st["_x2g_pack_order"].numpy(), order)
    info = st["_x2g_pack_info"].numpy().reshape(-1, 4)
    first = np.concatenate([[0], np.cumsum(deg)[:-1]])
    z = st["x"].numpy().reshape(-1)
    assert np.array_equal(info, np.stack([order, first[order], deg[order], z[order]], 1))
    # atoms without edges: a unit of their own (no rows)
    o2, p2, r2 = center_packs(np.array([0, 3, 0, 20, 5, 16, 1]))
    u2 = [o2[p2[u]:p2[u + 1]].tolist() for u in range(len(p2) - 1)]
    assert u2[-1] == [0, 2] and [3] in u2 and [5] in u2 and r2 == 20


def _center_packs_loop(deg, cap=16, max_members=16):
    """The best-fit-decreasing packing as a plain Python loop (round 5's data.center_packs, kept here as the
    checker of the native x2g_center_packs_host)."""
    deg = np.asarray(deg, dtype=np.int64)
    units, rows, free = [], [], [[] for _ in range(cap)]  # free[r]: open units with r rows left
    for a in np.argsort(-deg, kind="stable").tolist():
        d = int(deg[a])
        if d == 0:
            break
        if d < cap:
            for r in range(d, cap):  # the fullest open unit that takes it (the most recent on ties)
                if free[r]:
                    u = free[r].pop()
                    units[u].append(a)
                    rows[u] += d
                    if len(units[u]) < max_members:
                        free[r - d].append(u)
                    break
            else:
                free[cap - d].append(len(units))
                units.append([a])
                rows.append(d)
            continue
        units.append([a])
        rows.append(d)
    zero = np.flatnonzero(deg == 0).tolist()
    units += [zero[i:i + max_members] for i in range(0, len(zero), max_members)]
    rows += [0] * ((len(zero) + max_members - 1) // max_members)
    order = np.fromiter((a for u in units for a in u), dtype=np.int32, count=len(deg))
    packs = np.concatenate([[0], np.cumsum([len(u) for u in units])]).astype(np.int32)
    return order, packs, int(max(rows, default=0))


@pytest.mark.parametrize("case", ["s160", "s5a", "random", "ones", "zeros", "hubs", "empty", "members"])
def test_native_center_packs_equal_python_loop(case):
    """data.center_packs (native x2g_center_packs_host) == the Python best-fit loop, unit for unit: collated
    config-2 and S5A batches, random degrees with zeros and hubs, all-ones (the 16-member bound), no atoms."""
    from x2gnn.data import center_packs, collate
    from x2gnn.synth import synthetic_molecules

    rng = np.random.default_rng(7)
    if case in ("s160", "s5a"):
        b = collate(synthetic_molecules(64, "S160" if case == "s160" else "S5A", seed=3))
        deg = np.bincount(b.edge_index[0].numpy(), minlength=b.num_nodes)
    elif case == "random":
        deg = rng.integers(0, 40, size=3000)
    elif case == "ones":
        deg = np.ones(1000, dtype=np.int64)
    elif case == "zeros":
        deg = np.zeros(50, dtype=np.int64)
    elif case == "hubs":
        deg = np.concatenate([rng.integers(14, 70, size=200), rng.integers(0, 5, size=300)])
    elif case == "members":
        deg = rng.integers(1, 3, size=777)
    else:
        deg = np.zeros(0, dtype=np.int64)
    for cap, mm in ((16, 16), (8, 5)):
        o1, p1, r1 = center_packs(deg, cap, mm)
        o2, p2, r2 = _center_packs_loop(deg, cap, mm)
        assert np.array_equal(o1, o2) and np.array_equal(p1, p2) and r1 == r2, (case, cap, mm)
        assert o1.dtype == np.int32 and p1.dtype == np.int32


@pytest.mark.parametrize("host_schedule", [True, False])
def test_fast_collate_equals_pyg_from_data_list(monkeypatch, host_schedule):
    """collate (one numpy concatenation per key) == Batch.from_data_list over per-molecule Data objects (PyG
    2.1's collate restated, data.py), every key, dtype and the host metadata; with data.HOST_SCHEDULE False
    the center schedule is left to the device (and collate is cheaper)."""
    import time

    from x2gnn import data
    from x2gnn.synth import synthetic_molecules

    monkeypatch.setattr(data, "HOST_SCHEDULE", host_schedule)
    mols = synthetic_molecules(24, "S5A", seed=3)
    a = data.collate(mols)
    b = data.Batch.from_data_list([data.molecule_to_data(m) for m in mols])
    b._store["y"] = b._store["y"].to(torch.float32)
    assert list(a._store) == list(b._store)
    for k, va in a._store.items():
        vb = b._store[k]
        if torch.is_tensor(va):
            assert va.dtype == vb.dtype and torch.equal(va, vb), k
        else:
            assert va == vb, k
    for k in ("nodes", "edges", "triplets"):
        assert np.array_equal(a._meta[k], b._meta[k])
    assert ("_x2g_center_packs" in a._store) == host_schedule
    mols = synthetic_molecules(128, "S160", seed=1000)
    data.collate(mols)
    t0 = time.perf_counter()
    for _ in range(5):
        data.collate(mols)
    print(f"collate of 128 S160 molecules (host schedule {host_schedule}): {(time.perf_counter() - t0) / 5 * 1e3:.2f} ms")
