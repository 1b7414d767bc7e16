"""Host-side data formats and config-3 target preparation (train_ema.py:29-44)."""
import math
import os
import pickle

import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

from x2gnn import datasets as ds
from x2gnn.synth import radius_edges, triplet_count

XYZ_TWO = """3
-1.5
C 0.0 0.0 0.0
H 1.0 0.0 0.0
H 0.0 1.0 0.0
2
7.25
O 0.0 0.0 0.0
H 0.0 0.0 0.97
"""


def _write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_read_xyz_single_label(tmp_path):
    recs = ds.read_xyz(_write(tmp_path, "a.xyz", XYZ_TWO))
    assert len(recs) == 2
    assert recs[0].Z.tolist() == [6, 1, 1] and recs[1].Z.tolist() == [8, 1]
    assert recs[0].N.tolist() == [3] and recs[0].Label.tolist() == [-1.5] and recs[1].Label.tolist() == [7.25]
    assert recs[0].idx.tolist() == [0] and recs[1].idx.tolist() == [1]
    assert recs[0].R.dtype == torch.float32 and recs[1].R.shape == (2, 3)
    assert recs[1].atom.startswith("2\n7.25\nO 0.0 0.0 0.0\n")


def test_read_xyz_keeps_reference_quirks(tmp_path):
    # utils.py:57-61: the last molecule is appended only when the file's LAST line is an atom
    # line; blank lines in between are skipped
    assert len(ds.read_xyz(_write(tmp_path, "b.xyz", XYZ_TWO.replace("\n2\n", "\n\n2\n")))) == 2
    assert len(ds.read_xyz(_write(tmp_path, "c.xyz", XYZ_TWO + "\n"))) == 1


REF_AID = "/root/reference/raw/AID_kcal.xyz"


def _check_against_reference(recs, z, prefix):
    """x2gnn.datasets.read_xyz records == the reference's utils.read_xyz outputs stored in
    xyz_ref.npz (tests/golden/make_golden.py gen_xyz_ref ran the reference itself)."""
    import hashlib

    counts = z[prefix + "counts"]
    assert len(recs) == len(counts)
    assert [r.Z.shape[0] for r in recs] == counts.tolist()
    if len(recs):
        np.testing.assert_array_equal(np.concatenate([r.Z.numpy() for r in recs]), z[prefix + "z"])
        np.testing.assert_array_equal(np.concatenate([r.R.numpy().reshape(-1, 3) for r in recs]), z[prefix + "pos"])
        assert all(r.R.dtype == torch.float32 for r in recs if r.R.numel())
    for key, attr in (("label", "Label"), ("n", "N"), ("idx", "idx")):
        vals = [getattr(r, attr).numpy().reshape(-1) for r in recs]
        assert [len(v) for v in vals] == z[prefix + key + "_len"].tolist(), key
        if len(vals) and sum(len(v) for v in vals):
            np.testing.assert_array_equal(np.concatenate(vals).astype(z[prefix + key].dtype), z[prefix + key])
    if len(recs):
        assert str(recs[0].Label.dtype) == str(z[prefix + "label_dtype"][0])
    assert [hashlib.sha256(r.atom.encode()).hexdigest() for r in recs] == z[prefix + "atom_sha"].tolist()


def test_read_xyz_quirks_equal_reference(tmp_path):
    z = golden("xyz_ref.npz")
    for name in z["quirk_names"].tolist():
        recs = ds.read_xyz(_write(tmp_path, name + ".xyz", str(z[name + "_text"])))
        _check_against_reference(recs, z, name + "_")


@pytest.mark.skipif(not os.path.exists(REF_AID), reason="the reference's raw/AID_kcal.xyz is only in the build container")
def test_read_xyz_aid_equals_reference():
    """The whole AID_kcal.xyz (config 5's data) parsed here == the reference's own parse, and the
    committed aid_geom.npz (what the GPU box rebuilds config 5 from) is that parse."""
    z = golden("xyz_ref.npz")
    _check_against_reference(ds.read_xyz(REF_AID), z, "aid_")


def test_aid_geometry_fixture_is_reference_parse():
    z, aid = golden("xyz_ref.npz"), golden("aid_geom.npz")
    np.testing.assert_array_equal(aid["counts"], z["aid_counts"])
    np.testing.assert_array_equal(aid["z"].astype(np.int64), z["aid_z"])
    np.testing.assert_array_equal(aid["pos"], z["aid_pos"])
    np.testing.assert_array_equal(aid["label"], z["aid_label"])


def test_read_xyz_allprop(tmp_path):
    props = "\t".join(["1.5", "2.25", "-0.25", "0.1", "0.35", "19.0", "0.12", "-40.4", "-40.3", "-40.2",
                       "-40.5", "6.4*^-1"])
    text = f"2\n{props}\nC\t0.0\t0.0\t0.0\nH\t1.0\t1.5*^0\t0.0\n1\n{props}\nH\t0\t0\t0\n"
    recs = ds.read_xyz_allprop(_write(tmp_path, "q.xyz", text))
    assert len(recs) == 2
    assert recs[0].Label.shape == (1, 12) and recs[0].Label[0, 11].item() == pytest.approx(0.64)
    assert recs[0].R[1].tolist() == [1.0, 1.5, 0.0]
    with pytest.raises(ValueError):
        ds.read_xyz_allprop(_write(tmp_path, "bad.xyz", "1\n1.0 2.0\nH 0 0 0\n"))


def test_record_to_data_bonds_match_radius_edges():
    aid = golden("aid_geom.npz")
    counts = aid["counts"]
    off = np.concatenate([[0], np.cumsum(counts)])
    for m in (0, 7):
        z = aid["z"][off[m]:off[m + 1]].astype(np.int64)
        pos = aid["pos"][off[m]:off[m + 1]]
        rec = ds.MolRecord(atom="", R=torch.from_numpy(pos), Z=torch.from_numpy(z), N=torch.tensor([len(z)]),
                           Label=torch.tensor([0.0]), idx=torch.tensor([m]))
        d = ds.record_to_data(rec)
        ref = radius_edges(pos.astype(np.float64))
        # the float32 Gram-matrix distances (atom_graph.py:32-35) decide the same pairs as a
        # direct float64 distance for these geometries (no pair within rounding of the cutoff)
        np.testing.assert_array_equal(d.edge_index.numpy(), ref)
        assert d.edge_attr.shape == (ref.shape[1], 338) and d.edge_num == ref.shape[1]
        assert d._meta["triplets"][0] == triplet_count(ref, len(z))


def test_aid_geometry_fixture_shape():
    aid = golden("aid_geom.npz")
    c = aid["counts"]
    # 451 molecules, 60-146 atoms, ~83 on average
    assert len(c) == 451 and c.min() == 60 and c.max() == 146 and abs(c.mean() - 83.1) < 0.5
    assert set(np.unique(aid["z"]).tolist()) <= {1, 6, 7, 8, 9}


def test_load_collated_pyg_file():
    exp = golden("pyg_inmemory_v21.npz")
    data = ds.CollatedDataset.load(os.path.join(GOLDEN, "pyg_inmemory_v21.pt"))
    n = int(exp["n"])
    assert len(data) == n
    for k, v in data.slices.items():
        np.testing.assert_array_equal(v.numpy(), exp["slices_" + k])
    for i in range(n):
        d = data[i]
        for k in ("x", "edge_index", "edge_attr", "y", "atom_pos", "idx"):
            np.testing.assert_array_equal(d._store[k].numpy(), exp[f"{k}_{i}"])
        assert d.edge_num == int(exp[f"edge_num_{i}"][0])
        assert d._meta["triplets"][0] == triplet_count(exp[f"edge_index_{i}"], len(exp[f"x_{i}"]))
    with pytest.raises(IndexError):
        data[n]


def test_load_collated_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))

    p = tmp_path / "evil.pt"
    torch.save((Evil(), {"x": torch.arange(2)}), str(p), pickle_protocol=2)
    with pytest.raises(pickle.UnpicklingError):
        ds.load_collated(str(p))


def test_collated_molecules_form_a_batch():
    from x2gnn.data import Batch

    data = ds.CollatedDataset.load(os.path.join(GOLDEN, "pyg_inmemory_v21.pt"))
    b = Batch.from_data_list([data[i] for i in range(len(data))])
    exp = golden("pyg_inmemory_v21.npz")
    nodes = [len(exp[f"x_{i}"]) for i in range(len(data))]
    assert b.num_graphs == len(data) and b.y.shape == (len(data), 12)
    # PyG Batch increments edge_index by the running atom count
    np.testing.assert_array_equal(b.edge_index[:, :exp["edge_index_0"].shape[1]].numpy(), exp["edge_index_0"])
    np.testing.assert_array_equal(b.edge_index[:, exp["edge_index_0"].shape[1]:][:, :3].numpy(),
                                  exp["edge_index_1"][:, :3] + nodes[0])


@pytest.mark.parametrize("target", [0, 3, 7, 11])
def test_prepare_target_known_answer(target):
    data = ds.CollatedDataset.load(os.path.join(GOLDEN, "pyg_inmemory_v21.pt"))
    y12 = data.data.y.clone()
    z = data.data.x.clone()
    calib = ds.prepare_target(data, target)
    ref = ds.atom_reference_table()[target]
    off = data.slices["x"]
    for m in range(len(data)):
        mol_ref = sum(float(ref[int(a)]) for a in z[off[m]:off[m + 1]])
        want = float(y12[m, target]) - mol_ref
        if target in (2, 3, 4, 6, 7, 8, 9, 10):
            want *= 27.211385056
        assert float(data.data.y[m]) == pytest.approx(want, rel=1e-5)
    assert calib == (pytest.approx(1 / 0.04336414) if target in (2, 3, 4, 6, 7, 8, 9, 10) else 1)


def test_atom_reference_table():
    t = ds.atom_reference_table()
    assert t.shape == (12, 10) and torch.all(t[:7] == 0)
    assert t[7, 6].item() == pytest.approx(-37.846772) and t[11, 1].item() == pytest.approx(2.981)
    assert math.isnan(t[7, 0].item()) and math.isnan(t[10, 2].item())


def test_model_for_target_kinds():
    import x2gnn

    cfg = dict(conv_layers=1, sbf_dim=7, rbf_dim=6, in_channels=16, heads=2, embedding_size=16)
    for t in range(12):
        m = ds.model_for_target(t, cfg, device="cpu", pool_option="add")
        if t >= 6:
            assert type(m) is x2gnn.xgnn_poly
        else:
            assert type(m) is x2gnn.xgnn_poly_global
            assert m.fin_model.readouts[0].pool_option == "add"
