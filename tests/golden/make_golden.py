"""Generate the committed golden fixtures by running the REFERENCE (test infrastructure).

Run in the build container only (it imports /root/reference through ``ref_import``):

    python tests/golden/make_golden.py

Every fixture stores its inputs and the reference's outputs; weights are regenerated from a
seed by ``weights.seeded_value`` (see that module), so fixtures stay small.  Fixtures:

* ``triplets.npz``   — ``edge_graph.vertex_to_edge_2`` (edge_graph.py:12-30) on S160, S5A, a
                       3-molecule batch, the smallest AID_kcal molecule and a directed graph.
* ``basis.npz``/``basis_7x16.npz`` — ``poly_envelop`` (envelop.py:16-21), ``RadialBasis`` (radial_basis_layer.py:36-40)
                       and ``F_B_2D`` (angular_basis_layer.py:80-93) on a 2-molecule S160 batch.
* ``conv1.npz``      — one ``SBFTransformerConv`` (sbftransformer_conv.py:93-162), D=128 H=16,
                       per-triplet edge_attr, forward + backward for a seeded upstream gradient.
* ``model_small.npz``/``model_full.npz``/``model_global.npz`` — ``xgnn_poly`` / ``xgnn_poly_global``
                       forward energies and smooth-L1 parameter gradients (xgnn.py:38-75, model.py:38-54,
                       trainer.py:41-42).
* ``xyz_ref.npz``    — the reference's ``utils.read_xyz`` (utils.py:17-63) on raw/AID_kcal.xyz and on
                       small quirk files; ``aid_geom.npz`` is that same parse of AID_kcal.xyz as arrays.
"""
from __future__ import annotations

import hashlib
import os
import sys
import tempfile
import time
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))
sys.path.insert(0, HERE)

from ref_import import REF, import_reference  # noqa: E402
from weights import load_seeded  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.synth import molecule_from_geometry, read_xyz_molecules, synthetic_molecules  # noqa: E402

torch.set_num_threads(8)


def pack_batch(prefix, mols, out):
    b = collate(mols)
    out[prefix + "x"] = b.x.numpy()
    out[prefix + "atom_pos"] = b.atom_pos.numpy()
    out[prefix + "edge_index"] = b.edge_index.numpy().astype(np.int32)
    out[prefix + "edge_attr"] = b.edge_attr.numpy()
    out[prefix + "y"] = b.y.numpy()
    out[prefix + "nodes"] = b._meta["nodes"]
    out[prefix + "edges"] = b._meta["edges"]
    out[prefix + "triplets"] = b._meta["triplets"]
    return b


def directed_graph(seed=3, n=14, p=0.35):
    rng = np.random.default_rng(seed)
    adj = (rng.random((n, n)) < p) & ~np.eye(n, dtype=bool)
    src, dst = np.nonzero(adj)
    return np.stack([src, dst]).astype(np.int64), n


def gen_triplets(ref):
    out = {}
    cases = []
    cases.append(("s160", synthetic_molecules(1, "S160", seed=11)))
    cases.append(("s5a", synthetic_molecules(1, "S5A", seed=12)))
    cases.append(("batch3", synthetic_molecules(3, "S160", seed=13)))
    aid = read_xyz_molecules(os.path.join(REF, "raw/AID_kcal.xyz"))
    aid_small = min(aid, key=lambda m: len(m["x"]))
    cases.append(("aid", [aid_small]))
    names = []
    for name, mols in cases:
        b = collate(mols)
        ei, n = b.edge_index, b.num_nodes
        names.append(name)
        out[name + "_edge_index"] = ei.numpy().astype(np.int32)
        out[name + "_num_nodes"] = np.int64(n)
        _store_triplets(ref, out, name, ei, n)
    ei, n = directed_graph()
    names.append("directed")
    out["directed_edge_index"] = ei.astype(np.int32)
    out["directed_num_nodes"] = np.int64(n)
    _store_triplets(ref, out, "directed", torch.from_numpy(ei), n)
    out["cases"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "triplets.npz"), **out)


def _store_triplets(ref, out, name, ei, n):
    tri, j, i, k = ref.edge_graph.vertex_to_edge_2(ei.clone(), n)
    out[name + "_trip"] = np.asarray(tri).astype(np.int32)
    out[name + "_j"] = np.asarray(j).astype(np.int32)
    out[name + "_i"] = np.asarray(i).astype(np.int32)
    out[name + "_k"] = np.asarray(k).astype(np.int32)


def line_graph_inputs(ref, b):
    """The reference's featurisation steps (xgnn.py:39-65) for a collated batch."""
    pos, ei = b.atom_pos, b.edge_index
    d = torch.norm(pos[ei[0]] - pos[ei[1]], dim=1)
    tri, j, i, k = ref.edge_graph.vertex_to_edge_2(ei.clone(), b.num_nodes)
    ji = pos[i] - pos[j]
    jk = pos[k] - pos[j]
    cos_ = torch.sum(ji * jk, dim=1)
    sin_ = torch.norm(torch.cross(ji, jk, dim=1), dim=1)
    theta = torch.atan2(sin_, cos_)
    return d, tri, theta, (j, i, k)


def gen_basis(ref):
    out = {}
    b = pack_batch("", synthetic_molecules(2, "S160", seed=21), out)
    d, tri, theta, _ = line_graph_inputs(ref, b)
    env = ref.envelop.poly_envelop(cutoff=5.0, exponent=5)
    sbf_layer = ref.angular_basis_layer.F_B_2D(7, 6, 5.0, 5)
    rbf_layer = ref.radial_basis_layer.RadialBasis(cutoff=5.0, embedding_size=6)
    with torch.no_grad():
        out["dist"] = d.numpy()
        out["theta"] = theta.numpy()
        out["trip"] = tri.numpy().astype(np.int32)
        out["env"] = env(d).numpy()
        out["sbf"] = sbf_layer(d, theta, tri[0]).numpy()
        out["rbf"] = (rbf_layer(d) * env(d)[:, None]).numpy()
        # envelope known answers (x = d/5): 1/x - 28x^5 + 48x^6 - 21x^7
        probe = torch.tensor([0.5, 1.0, 2.5, 4.999, 5.0])
        out["env_probe_d"] = probe.numpy()
        out["env_probe"] = env(probe).numpy()
    np.savez_compressed(os.path.join(HERE, "basis.npz"), **out)


def gen_basis_7x16(ref):
    """basis_7x16.npz: F_B_2D(7, 16) (the reference's default xgnn_poly basis, xgnn.py:16) and
    RadialBasis(16) on the basis.npz batch."""
    out = {}
    b = pack_batch("", synthetic_molecules(2, "S160", seed=21), out)
    d, tri, theta, _ = line_graph_inputs(ref, b)
    env = ref.envelop.poly_envelop(cutoff=5.0, exponent=5)
    sbf_layer = ref.angular_basis_layer.F_B_2D(7, 16, 5.0, 5)
    rbf_layer = ref.radial_basis_layer.RadialBasis(cutoff=5.0, embedding_size=16)
    with torch.no_grad():
        out["dist"] = d.numpy()
        out["theta"] = theta.numpy()
        out["trip"] = tri.numpy().astype(np.int32)
        out["sbf"] = sbf_layer(d, theta, tri[0]).numpy()
        out["rbf"] = (rbf_layer(d) * env(d)[:, None]).numpy()
    np.savez_compressed(os.path.join(HERE, "basis_7x16.npz"), **out)


def gen_conv1(ref):
    out = {}
    b = pack_batch("", synthetic_molecules(1, "S160", seed=31), out)
    d, tri, theta, _ = line_graph_inputs(ref, b)
    sbf_layer = ref.angular_basis_layer.F_B_2D(7, 6, 5.0, 5)
    env = ref.envelop.poly_envelop(cutoff=5.0, exponent=5)
    rbf_layer = ref.radial_basis_layer.RadialBasis(cutoff=5.0, embedding_size=6)
    with torch.no_grad():
        sbf = sbf_layer(d, theta, tri[0])
        rbf = rbf_layer(d) * env(d)[:, None]
    E, T = d.shape[0], tri.shape[1]
    g = torch.Generator().manual_seed(7)
    x = torch.randn(E, 128, generator=g).requires_grad_(True)
    ea = torch.randn(T, 128, generator=g).requires_grad_(True)
    up = torch.randn(E, 128, generator=g)
    conv = ref.sbftransformer_conv.SBFTransformerConv(in_channels=128, out_channels=8, heads=16, sbf_dim=42,
                                                      rbf_dim=6, dropout=0, edge_dim=128)
    load_seeded(conv, seed=101)
    y = conv(sbf=sbf, rbf=rbf, x=x, edge_index=tri, edge_attr=ea)
    (y * up).sum().backward()
    out.update(sbf=sbf.numpy(), rbf=rbf.numpy(), trip=tri.numpy().astype(np.int32), conv_x=x.detach().numpy(),
               conv_edge_attr=ea.detach().numpy(), upstream=up.numpy(), out=y.detach().numpy(),
               grad_x=x.grad.numpy(), grad_edge_attr=ea.grad.numpy(), weight_seed=np.int64(101))
    for n, p in conv.named_parameters():
        out["grad." + n] = p.grad.numpy()
    np.savez_compressed(os.path.join(HERE, "conv1.npz"), **out)


def gen_model(ref, fname, kind, cfg, n_mol, seed_mol, seed_w, grads="all", pool_option="mean", shape="S160",
              mols=None):
    out = {}
    if mols is None:
        mols = synthetic_molecules(n_mol, shape, seed=seed_mol)
    b = pack_batch("", mols, out)
    if kind == "poly":
        model = ref.xgnn.xgnn_poly(device="cpu", **cfg)
    else:
        model = ref.xgnn.xgnn_poly_global(device="cpu", pool_option=pool_option, **cfg)
    load_seeded(model, seed=seed_w)
    t0 = time.time()
    res = model(b)
    loss = torch.nn.functional.smooth_l1_loss(res, b.y)
    loss.backward()
    print(f"{fname}: fwd+bwd {time.time() - t0:.2f}s  E={b.edge_index.shape[1]}  T={int(b._meta['triplets'].sum())}")
    out["energies"] = res.detach().numpy()
    out["loss"] = np.float32(loss.item())
    out["weight_seed"] = np.int64(seed_w)
    out["cfg_keys"] = np.array(list(cfg.keys()))
    out["cfg_vals"] = np.array(list(cfg.values()))
    out["kind"] = np.array(kind)
    out["pool_option"] = np.array(pool_option)
    out["param_names"] = np.array([n for n, _ in model.named_parameters()])
    out["param_shapes"] = np.array([str(tuple(p.shape)) for _, p in model.named_parameters()])
    out["state_keys"] = np.array(list(model.state_dict().keys()))
    out["emb_after"] = model.emb_block.embedding.weight.detach().numpy().copy()
    for n, p in model.named_parameters():
        gr = p.grad
        out["gnorm." + n] = np.float64(0.0 if gr is None else gr.double().norm().item())
        if gr is not None and (grads == "all" or n in grads):
            out["grad." + n] = gr.numpy()
    np.savez_compressed(os.path.join(HERE, fname), **out)


def _reference_read_xyz():
    """The reference's own ``utils.read_xyz`` (utils.py:17-63).  utils.py imports ``pyscf.lib``
    at line 2 and never uses it; pyscf is absent here, so an empty stand-in module satisfies the
    import (nothing else is patched)."""
    if "pyscf" not in sys.modules:
        pyscf = types.ModuleType("pyscf")
        pyscf.lib = types.ModuleType("pyscf.lib")
        sys.modules["pyscf"], sys.modules["pyscf.lib"] = pyscf, pyscf.lib
    import utils  # noqa: E402  (/root/reference/utils.py, on sys.path via import_reference)
    return utils.read_xyz


# small files that exercise utils.py's quirks (blank lines skipped; the last molecule is kept
# only when the file's last line is an atom line); the reference's results on them are pinned
XYZ_QUIRKS = {
    "two": "3\n-1.5\nC 0.0 0.0 0.0\nH 1.0 0.0 0.0\nH 0.0 1.0 0.0\n2\n7.25\nO 0.0 0.0 0.0\nH 0.0 0.0 0.97\n",
    "blank_between": "3\n-1.5\nC 0.0 0.0 0.0\nH 1.0 0.0 0.0\nH 0.0 1.0 0.0\n\n2\n7.25\nO 0.0 0.0 0.0\nH 0.0 0.0 0.97\n",
    "trailing_blank": "3\n-1.5\nC 0.0 0.0 0.0\nH 1.0 0.0 0.0\nH 0.0 1.0 0.0\n2\n7.25\nO 0.0 0.0 0.0\nH 0.0 0.0 0.97\n\n",
    "int_label": "1\n4\nH 0.5 0.25 0.125\n2\n-3.0\nN 1 2 3\nF 4 5 6.5\n",
}


def _pack_records(recs, prefix, out):
    out[prefix + "counts"] = np.array([r.Z.shape[0] for r in recs], dtype=np.int32)
    out[prefix + "z"] = (np.concatenate([r.Z.numpy() for r in recs]) if recs else np.zeros(0)).astype(np.int64)
    out[prefix + "pos"] = (np.concatenate([r.R.numpy().reshape(-1, 3) for r in recs]) if recs
                           else np.zeros((0, 3))).astype(np.float32)
    for key, attr, dt in (("label", "Label", np.float64), ("n", "N", np.int64), ("idx", "idx", np.int64)):
        vals = [getattr(r, attr).numpy().reshape(-1) for r in recs]  # ragged: a list per record
        out[prefix + key] = (np.concatenate(vals) if vals else np.zeros(0)).astype(dt)
        out[prefix + key + "_len"] = np.array([len(v) for v in vals], dtype=np.int64)
    out[prefix + "atom_sha"] = np.array([hashlib.sha256(r.atom.encode()).hexdigest() for r in recs])
    out[prefix + "label_dtype"] = np.array([str(recs[0].Label.dtype) if recs else ""])


def gen_xyz_ref(ref):
    """xyz_ref.npz: the reference's utils.read_xyz run here on raw/AID_kcal.xyz (config 5's
    data) and on the XYZ_QUIRKS texts: Z / positions / labels / counts / idx and a hash of each
    record's xyz text, so tests/test_datasets.py pins x2gnn.datasets.read_xyz to it."""
    read_xyz = _reference_read_xyz()
    out = {}
    _pack_records(read_xyz(os.path.join(REF, "raw/AID_kcal.xyz")), "aid_", out)
    with tempfile.TemporaryDirectory() as tmp:
        for name, text in XYZ_QUIRKS.items():
            p = os.path.join(tmp, name + ".xyz")
            with open(p, "w") as f:
                f.write(text)
            _pack_records(read_xyz(p), name + "_", out)
    out["quirk_names"] = np.array(list(XYZ_QUIRKS))
    for name, text in XYZ_QUIRKS.items():
        out[name + "_text"] = np.array(text)
    np.savez_compressed(os.path.join(HERE, "xyz_ref.npz"), **out)
    print(f"xyz_ref.npz: {len(out['aid_counts'])} AID molecules + {len(XYZ_QUIRKS)} quirk files")


def gen_aid_geometry(ref):
    """aid_geom.npz: every molecule of raw/AID_kcal.xyz (config 5's data) as Z / positions /
    label arrays, parsed by the reference's own utils.read_xyz (utils.py:17-63), so the GPU box
    (where /root/reference does not exist) can rebuild the molecules."""
    recs = _reference_read_xyz()(os.path.join(REF, "raw/AID_kcal.xyz"))
    np.savez_compressed(os.path.join(HERE, "aid_geom.npz"),
                        counts=np.array([r.Z.shape[0] for r in recs], dtype=np.int32),
                        z=np.concatenate([r.Z.numpy() for r in recs]).astype(np.int8),
                        pos=np.concatenate([r.R.numpy() for r in recs]).astype(np.float32),
                        label=np.array([float(r.Label.reshape(-1)[0]) for r in recs]))
    print(f"aid_geom.npz: {len(recs)} molecules")


SMALL = dict(conv_layers=2, sbf_dim=7, rbf_dim=6, in_channels=32, heads=4, embedding_size=32)
FULL = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)
SEL = ["fin_model.convs.0.lin_sbf.weight", "fin_model.convs.3.lin_query.weight",
       "fin_model.convs.1.lin_edge.weight", "emb_block.embedding.weight", "rbf_layer.frequencies",
       "fin_model.readouts.2.lin_rbf.weight", "fin_model.edgenn.0.weight", "mat_trans.weight"]
SEL_CONV = [f"fin_model.convs.{i}.{lin}.{p}" for i in (0, 3)
            for lin in ("lin_key", "lin_value", "lin_query", "lin_skip", "lin_sbf", "lin_edge", "lin_rbf")
            for p in ("weight", "bias")]


def aid_molecules(k, seed=0):
    """The k smallest AID_kcal molecules (config 5 geometry, seeded synthetic edge features)."""
    from x2gnn.datasets import read_xyz
    recs = sorted(read_xyz(os.path.join(REF, "raw/AID_kcal.xyz")), key=lambda r: r.Z.shape[0])[:k]
    return [molecule_from_geometry(r.Z.numpy(), r.R.numpy().astype(np.float64), 5.0,
                                   np.random.default_rng(1000 * seed + i + 17), y=float(r.Label.reshape(-1)[0]))
            for i, r in enumerate(recs)]


GENERATORS = {
    "triplets": lambda ref: gen_triplets(ref),
    "basis": lambda ref: gen_basis(ref),
    "basis_7x16": lambda ref: gen_basis_7x16(ref),
    "conv1": lambda ref: gen_conv1(ref),
    "model_small": lambda ref: gen_model(ref, "model_small.npz", "poly", SMALL, n_mol=4, seed_mol=41, seed_w=201),
    "model_full": lambda ref: gen_model(ref, "model_full.npz", "poly", FULL, n_mol=2, seed_mol=42, seed_w=202,
                                        grads=SEL),
    "model_global": lambda ref: gen_model(ref, "model_global.npz", "global", SMALL, n_mol=4, seed_mol=43,
                                          seed_w=203, pool_option="mean"),
    "model_s5a": lambda ref: gen_model(ref, "model_s5a.npz", "poly", SMALL, n_mol=2, seed_mol=44, seed_w=204,
                                       shape="S5A"),
    # config 3: the MolWise model with the other pool option, at full width
    "model_global_add": lambda ref: gen_model(ref, "model_global_add.npz", "global", FULL, n_mol=3, seed_mol=45,
                                              seed_w=205, pool_option="add", grads=SEL[:5]),
    # config 5: real AID geometry (the two smallest molecules), full width
    "model_aid": lambda ref: gen_model(ref, "model_aid.npz", "poly", FULL, n_mol=1, seed_mol=0, seed_w=206,
                                       grads=SEL, mols=aid_molecules(2)),
    # config-2 width on the physical 5 A geometry (degrees up to 17): the shipped center-atom attention
    # kernels (D = 128 only) against the reference with per-element gradients of every conv projection
    # of two layers (lin_key / lin_value / lin_sbf / lin_rbf carry the center backward's dk, dv, G)
    "model_s5a_full": lambda ref: gen_model(ref, "model_s5a_full.npz", "poly", FULL, n_mol=2, seed_mol=46,
                                            seed_w=207, shape="S5A", grads=SEL + SEL_CONV),
    "aid_geom": lambda ref: gen_aid_geometry(ref),
    "xyz_ref": lambda ref: gen_xyz_ref(ref),
}


def main():
    names = sys.argv[1:] or list(GENERATORS)
    ref = import_reference()
    for n in names:
        GENERATORS[n](ref)


if __name__ == "__main__":
    main()
