"""Synthetic QM9-shaped molecules (host side, numpy).

QM9 itself is not available offline (the reference ships only the last part of a split
archive, and its 338-wide edge features come from pyscf integrals, scf.py:50-118), so the
benchmark and the parity tests run on synthetic molecules of the same shape:

* geometry: ``n_heavy`` heavy atoms grown as a random tree (bond ``1.5*s`` Angstrom, minimum
  separation ``1.3*s``), then ``n_h`` hydrogens at ``1.09*s`` from a random heavy atom
  (minimum separation ``0.9*s``).  ``s=1.8`` gives the "S160" shape (~18 atoms, ~160
  directed edges, ~1460 triplets per molecule); ``s=1.0`` the physical 5 A "S5A" shape.
* element mix C:N:O:F ~ 72:11:16:1 (QM9-like), hydrogens Z=1.
* edges: every ordered pair with 0 < d < cutoff, enumerated row-major exactly like
  ``np.argwhere`` in the reference's ``gen_bonds_mini`` (atom_graph.py:42-45), so the edge
  list is sorted by source atom then destination atom.
* edge_attr ~ N(0, 0.1^2), float32 [E, 338] (stands in for the pyscf features).

AID_kcal.xyz (the reference's raw/AID_kcal.xyz, config 5) is read by :func:`read_xyz_molecules`
with the same grammar as the reference's utils.py:17-63 (count line, label line, ``El x y z``).
"""
from __future__ import annotations

import numpy as np

ATOM_NUMBER = {"H": 1, "C": 6, "N": 7, "O": 8, "F": 9}
EDGE_FEATURES = 338  # scf.py: 2 x 13 x 13 symmetry-adapted blocks

SHAPES = {"S160": 1.8, "S5A": 1.0}


def _unit(rng):
    v = rng.normal(size=3)
    return v / np.linalg.norm(v)


def random_geometry(rng, scale: float, n_heavy: int = 9, n_h: int = 9):
    """Return (Z int64[n], pos float64[n,3]) for one synthetic molecule."""
    heavy_z = np.array([6, 7, 8, 9])
    heavy_p = np.array([0.72, 0.11, 0.16, 0.01])
    pos = [np.zeros(3)]
    while len(pos) < n_heavy:
        parent = pos[rng.integers(len(pos))]
        cand = parent + 1.5 * scale * _unit(rng)
        if min(np.linalg.norm(cand - p) for p in pos) >= 1.3 * scale - 1e-9:
            pos.append(cand)
    n_heavy_placed = len(pos)
    while len(pos) < n_heavy_placed + n_h:
        parent = pos[rng.integers(n_heavy_placed)]
        cand = parent + 1.09 * scale * _unit(rng)
        if min(np.linalg.norm(cand - p) for p in pos) >= 0.9 * scale - 1e-9:
            pos.append(cand)
    z = np.concatenate([rng.choice(heavy_z, size=n_heavy, p=heavy_p),
                        np.ones(n_h, dtype=np.int64)]).astype(np.int64)
    return z, np.asarray(pos)


def radius_edges(pos: np.ndarray, cutoff: float = 5.0) -> np.ndarray:
    """Directed edges 0 < d < cutoff in row-major (src, dst) order, int64 [2, E]."""
    diff = pos[:, None, :] - pos[None, :, :]
    d = np.sqrt((diff * diff).sum(-1))
    adj = (d < cutoff) & (d > 0)
    src, dst = np.nonzero(adj)  # row-major == np.argwhere order
    return np.stack([src, dst]).astype(np.int64)


def triplet_count(edge_index: np.ndarray, num_nodes: int) -> int:
    """Number of line-graph edges: sum over e=(a->b) of |N_out(b) \\ {a}|."""
    src, dst = edge_index
    deg = np.bincount(src, minlength=num_nodes)
    n = deg[dst].sum()
    # subtract one for each e=(a->b) whose reverse (b->a) exists
    key = src.astype(np.int64) * num_nodes + dst
    rev = dst.astype(np.int64) * num_nodes + src
    n -= np.isin(rev, key).sum()
    return int(n)


def make_molecule(rng, scale: float, cutoff: float = 5.0, feat_rng=None, with_attr=True):
    z, pos = random_geometry(rng, scale)
    return molecule_from_geometry(z, pos, cutoff, feat_rng if feat_rng is not None else rng,
                                  with_attr=with_attr)


def molecule_from_geometry(z, pos, cutoff=5.0, feat_rng=None, with_attr=True, y=None):
    pos = np.asarray(pos, dtype=np.float64)
    ei = radius_edges(pos, cutoff)
    mol = {
        "x": np.asarray(z, dtype=np.int64),
        "atom_pos": pos.astype(np.float32),
        "edge_index": ei,
        "edge_num": ei.shape[1],
        "triplet_num": triplet_count(ei, len(z)),
    }
    if with_attr:
        frng = feat_rng if feat_rng is not None else np.random.default_rng(0)
        mol["edge_attr"] = (0.1 * frng.standard_normal((ei.shape[1], EDGE_FEATURES))).astype(np.float32)
    mol["y"] = np.float32(y if y is not None else 0.0)
    return mol


def synthetic_molecules(n: int, shape: str = "S160", seed: int = 0, cutoff: float = 5.0):
    """``n`` synthetic molecules (list of dicts) of the named shape, deterministic in ``seed``."""
    scale = SHAPES[shape]
    geo = np.random.default_rng(seed)
    mols = []
    for m in range(n):
        feat = np.random.default_rng(1000 * seed + m + 17)
        mol = make_molecule(geo, scale, cutoff, feat_rng=feat)
        mol["y"] = np.float32(feat.normal())
        mols.append(mol)
    return mols


def read_xyz_molecules(path: str, limit: int | None = None, cutoff: float = 5.0, seed: int = 0):
    """Parse a multi-molecule xyz file (count / label / ``El x y z`` lines) into molecules.

    Grammar follows the reference's ``read_xyz`` (utils.py:17-63); the label line is the
    target value.  Edge features are synthetic (pyscf is not available).
    """
    mols = []
    with open(path) as f:
        lines = [ln for ln in f.read().split("\n")]
    i = 0
    while i < len(lines):
        s = lines[i].strip()
        if not s:
            i += 1
            continue
        count = int(s)
        label = float(lines[i + 1].split()[0])
        z, pos = [], []
        for ln in lines[i + 2:i + 2 + count]:
            el, x, y, zz = ln.split()[:4]
            z.append(ATOM_NUMBER[el])
            pos.append((float(x), float(y), float(zz)))
        feat = np.random.default_rng(1000 * seed + len(mols) + 17)
        mols.append(molecule_from_geometry(np.array(z), np.array(pos), cutoff, feat, y=label))
        i += 2 + count
        if limit is not None and len(mols) >= limit:
            break
    return mols


def molecules_from_geometry_file(path: str, indices=None, cutoff: float = 5.0, seed: int = 0):
    """Molecules from a geometry archive (``counts`` int [M], ``z`` [sum], ``pos`` [sum, 3],
    optional ``label`` [M]; e.g. tests/golden/aid_geom.npz, the reference's raw/AID_kcal.xyz as
    arrays) with seeded synthetic edge features; ``indices`` selects molecules (default all)."""
    arc = np.load(path, allow_pickle=False)
    counts = arc["counts"].astype(np.int64)
    off = np.concatenate([[0], np.cumsum(counts)])
    labels = arc["label"] if "label" in arc.files else np.zeros(len(counts))
    idx = range(len(counts)) if indices is None else indices
    mols = []
    for j, m in enumerate(idx):
        z = arc["z"][off[m]:off[m + 1]].astype(np.int64)
        pos = arc["pos"][off[m]:off[m + 1]].astype(np.float64)
        feat = np.random.default_rng(1000 * seed + j + 17)
        mols.append(molecule_from_geometry(z, pos, cutoff, feat, y=float(labels[m])))
    return mols
