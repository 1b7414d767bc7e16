"""The reference's data formats and target preparation.

* ``read_xyz`` — the single-label xyz grammar of utils.py:17-63 (count line, one label line,
  ``El x y z`` lines) into :class:`MolRecord` (utils.py:6-15's ``Mol_Object``), with the same
  quirks: a line with one token is a count when it parses as an int and a label when it parses
  as a float, blank lines are skipped, the record list starts at the second count line's
  predecessor (``mol_list[1:]``), and the last molecule is only kept when the file's last
  line is an atom line.
* ``read_xyz_allprop`` — the 12-property QM9 file written by datapre.ipynb cell 3 (count line,
  12 tab-separated properties, tab-separated ``El x y z`` lines; ``*^`` exponents already
  rewritten to ``E``) that qm9_allprop.py:50 reads through ``utils.read_xyz_allprop`` (that
  function is not in the reference tree; this restates the format the notebook writes).
  ``Label`` is [1, 12] so a collate stacks it to [M, 12] (train_ema.py:32 indexes ``y[:, t]``).
* ``record_to_data`` — qm9_allprop.py:11-19's ``mapping`` minus the pyscf features: the
  distance matrix of atom_graph.py:32-35 (float32 Gram form) and ``gen_bonds_mini``'s
  ``argwhere((D < cutoff) & D != 0)`` (atom_graph.py:42-45).  ``edge_attr`` must be supplied
  (pyscf is not available); :func:`synthetic_edge_attr` gives the seeded stand-in.
* ``load_collated`` — a PyG ``InMemoryDataset`` processed file (qm9_allprop.py:58,
  ``torch.save(self.collate(datas), ...)`` = a pickled ``(Data, slices)`` under PyG 2.1.0) read
  with ``torch.load(weights_only=True)``: the PyG classes the pickle names are allow-listed as
  inert stand-ins (nothing from the file is executed), and the tensors are taken out of the
  stand-in's storage mapping.  The PyG >= 2.4 layout ``(data_dict, slices, sizes, cls)`` is
  accepted too.  :class:`CollatedDataset` mirrors ``InMemoryDataset``'s ``data`` / ``slices`` /
  ``len`` / ``__getitem__`` (per-molecule slices, ``edge_index`` not incremented, as PyG's
  ``collate(increment=False)`` stores it).
* ``prepare_target`` — train_ema.py:29-38: pick column ``target``, subtract the per-molecule sum
  of atomic reference energies, convert Hartree -> eV for targets 2,3,4,6..10, and return the
  ``print_calibration`` factor; ``model_for_target`` — train_ema.py:41-44 (targets 6-11 are
  ``xgnn_poly``/AtomWise, 0-5 ``xgnn_poly_global``/MolWise).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from .data import Data
from .synth import EDGE_FEATURES, triplet_count

ATOM_NUMBER = {"H": 1, "C": 6, "N": 7, "O": 8, "F": 9}  # utils.py:19
LABELS = {0: "dipole", 1: "polarizability", 2: "HOMO", 3: "LUMO", 4: "GAP", 5: "spatial extent", 6: "zpve",
          7: "U0", 8: "U", 9: "H", 10: "G", 11: "Cv"}  # train_ema.py:9
HARTREE_TO_EV = 27.211385056  # train_ema.py:35
EV_TARGETS = (2, 3, 4, 6, 7, 8, 9, 10)  # train_ema.py:34
ATOMWISE_TARGETS = (6, 7, 8, 9, 10, 11)  # train_ema.py:41
PRINT_CALIBRATION_EV = 1 / 0.04336414  # train_ema.py:36


def atom_reference_table() -> torch.Tensor:
    """[12, 10] per-element reference energies (train_ema.py:10-21): rows 7-11 carry H, C, N, O,
    F values (NaN for the other element slots, so a molecule with any other element gets a NaN
    target, as in the reference); rows 0-6 are zero."""
    nan = math.nan
    ref = torch.zeros(12, 10)
    rows = {
        7: [-0.500273, -37.846772, -54.583861, -75.064579, -99.718730],
        8: [-0.498857, -37.845355, -54.582445, -75.063163, -99.717314],
        9: [-0.497912, -37.844411, -54.581501, -75.062219, -99.716370],
        10: [-0.510927, -37.861317, -54.598897, -75.079532, -99.733544],
        11: [2.981, 2.981, 2.981, 2.981, 2.981],
    }
    for t, (h, c, n, o, f) in rows.items():
        ref[t] = torch.tensor([nan, h, nan, nan, nan, nan, c, n, o, f])
    return ref


@dataclass
class MolRecord:
    """utils.py:6-15 ``Mol_Object``: xyz text, R [n,3] float32, Z [n], N [1], Label, idx."""
    atom: str
    R: torch.Tensor
    Z: torch.Tensor
    N: torch.Tensor
    Label: torch.Tensor
    idx: torch.Tensor
    force: torch.Tensor | None = field(default=None)


def _record(atom, R, Z, N, y, idx):
    return MolRecord(atom=atom, R=torch.tensor(R) if R else torch.zeros(0, 3), Z=torch.tensor(Z, dtype=torch.int64),
                     N=torch.tensor(N, dtype=torch.int64), Label=torch.tensor(y), idx=torch.tensor(idx, dtype=torch.int64))


def _one_token_kind(tok: str):
    """utils.py:35-51 branches on ``type(eval(line))``: int -> count line, float -> label line."""
    try:
        return "count", int(tok)
    except ValueError:
        return "label", float(tok)


def read_xyz(path: str) -> list[MolRecord]:
    """utils.py:17-63 restated (see the module docstring for the quirks kept)."""
    with open(path) as f:
        lines = f.readlines()
    out = []
    atom, R, N, Z, y, idx = "", [], [], [], [], [0]
    counter = 0
    end = len(lines) - 1
    for i, line in enumerate(lines):
        if line == "\n":
            continue
        toks = line.split()
        if len(toks) == 1:
            kind, val = _one_token_kind(toks[0])
            if kind == "count":
                out.append(_record(atom, R, Z, N, y, idx))
                atom, R, N, Z, y, idx = "", [], [], [], [], [counter]
                counter += 1
                atom += line
                N.append(val)
            else:
                y.append(val)
                atom += line
        elif len(toks) == 4:
            atom += f"{toks[0]} {toks[1]} {toks[2]} {toks[3]}\n"
            R.append([float(v) for v in toks[1:]])
            Z.append(ATOM_NUMBER[toks[0]])
            if i == end:
                out.append(_record(atom, R, Z, N, y, idx))
    return out[1:]


def read_xyz_allprop(path: str, num_props: int = 12) -> list[MolRecord]:
    """The datapre.ipynb cell-3 format (count / ``num_props`` properties / ``El x y z``)."""
    with open(path) as f:
        lines = [ln for ln in f.read().split("\n")]
    out, i = [], 0
    while i < len(lines):
        s = lines[i].strip()
        if not s:
            i += 1
            continue
        count = int(s)
        props = [float(v.replace("*^", "E")) for v in lines[i + 1].split()]
        if len(props) != num_props:
            raise ValueError(f"line {i + 2}: expected {num_props} properties, got {len(props)}")
        atom = lines[i] + "\n" + lines[i + 1] + "\n"
        R, Z = [], []
        for ln in lines[i + 2:i + 2 + count]:
            toks = ln.replace("*^", "E").split()
            if len(toks) != 4:
                raise ValueError(f"bad atom line {ln!r}")
            Z.append(ATOM_NUMBER[toks[0]])
            R.append([float(v) for v in toks[1:]])
            atom += " ".join(toks) + "\n"
        out.append(_record(atom, R, Z, [count], [props], [len(out)]))
        i += 2 + count
    return out


def distance_matrix(R: torch.Tensor) -> torch.Tensor:
    """atom_graph.py:32-35: relu(sqrt(diag(G) + diag(G)^T - 2G)) with G = R R^T (float32; the
    diagonal may come out NaN from a tiny negative, which the edge test below rejects)."""
    R = R.to(torch.float32)
    G = R @ R.T
    H = torch.diag(G).repeat(R.shape[0], 1)
    return torch.relu((H + H.T - 2 * G) ** 0.5)


def bonds(D: torch.Tensor, cutoff: float = 5.0) -> torch.Tensor:
    """atom_graph.py:42-45 ``gen_bonds_mini``: int64 [2, E] of (D < cutoff) & D != 0, row-major."""
    adj = (D < cutoff) & D.bool()
    return torch.from_numpy(np.argwhere(adj.numpy()).T.copy()).to(torch.int64)


def synthetic_edge_attr(num_edges: int, seed: int) -> torch.Tensor:
    """Seeded N(0, 0.1^2) stand-in for scf.py's 338 pyscf features (see synth.py)."""
    rng = np.random.default_rng(seed)
    return torch.from_numpy((0.1 * rng.standard_normal((num_edges, EDGE_FEATURES))).astype(np.float32))


def record_to_data(rec: MolRecord, edge_attr: torch.Tensor | None = None, cutoff: float = 5.0,
                   feat_seed: int | None = None) -> Data:
    """qm9_allprop.py:11-19 ``mapping`` with ``edge_attr`` given or seeded (see module doc)."""
    ei = bonds(distance_matrix(rec.R), cutoff)
    if edge_attr is None:
        edge_attr = synthetic_edge_attr(ei.shape[1], int(rec.idx.reshape(-1)[0]) if feat_seed is None else feat_seed)
    if edge_attr.shape[0] != ei.shape[1]:
        raise ValueError(f"edge_attr has {edge_attr.shape[0]} rows for {ei.shape[1]} edges")
    d = Data(x=rec.Z.clone(), edge_index=ei, edge_attr=edge_attr.to(torch.float32), y=rec.Label.clone(),
             edge_num=int(ei.shape[1]), idx=rec.idx.clone(), atom_pos=rec.R.to(torch.float32))
    object.__setattr__(d, "_meta", {"nodes": np.array([rec.Z.shape[0]]), "edges": np.array([ei.shape[1]]),
                                    "triplets": np.array([triplet_count(ei.numpy(), rec.Z.shape[0])])})
    return d


# ---------------------------------------------------------------------------------- PyG .pt files
class _Inert:
    """Allow-listed stand-in for a PyG class named in a pickle: keeps whatever state/args the
    pickle hands it and runs no code of its own beyond that."""

    def __init__(self, *args, **kwargs):
        self.__dict__["_args"] = args

    def __setstate__(self, state):
        if isinstance(state, tuple) and len(state) == 2:  # (dict state, slot state)
            for part in state:
                if isinstance(part, dict):
                    self.__dict__.update(part)
        elif isinstance(state, dict):
            self.__dict__.update(state)
        else:
            self.__dict__["_state"] = state


_PYG_NAMES = [
    "torch_geometric.data.data.Data",
    "torch_geometric.data.data.DataTensorAttr",
    "torch_geometric.data.data.DataEdgeAttr",
    "torch_geometric.data.storage.GlobalStorage",
    "torch_geometric.data.storage.BaseStorage",
    "torch_geometric.data.storage.NodeStorage",
    "torch_geometric.data.storage.EdgeStorage",
    "torch_geometric.data.feature_store.TensorAttr",
    "torch_geometric.data.graph_store.EdgeAttr",
    "torch_geometric.data.graph_store.EdgeLayout",
    "torch_geometric.data.in_memory_dataset.InMemoryDataset",
]


def _stand_ins():
    out = []
    for name in _PYG_NAMES:
        cls = type(name.rsplit(".", 1)[1], (_Inert,), {"__module__": "x2gnn.datasets._pyg"})
        out.append((cls, name))
    return out


def _mapping_of(obj):
    """Tensors of a PyG Data stand-in (``_store`` -> ``_mapping``) or of a plain dict."""
    if isinstance(obj, dict):
        return dict(obj)
    d = getattr(obj, "__dict__", {})
    store = d.get("_store")
    if store is not None:
        sd = store.__dict__ if hasattr(store, "__dict__") else {}
        if "_mapping" in sd:
            return dict(sd["_mapping"])
        return {k: v for k, v in sd.items() if not k.startswith("_")}
    if "_mapping" in d:
        return dict(d["_mapping"])
    raise ValueError(f"cannot find the tensor mapping of {type(obj).__name__}")


def load_collated(path: str):
    """Read an ``InMemoryDataset`` processed file; returns (mapping of concatenated tensors,
    slices dict).  Only ``torch.load(weights_only=True)`` runs on the file."""
    with torch.serialization.safe_globals(_stand_ins()):
        obj = torch.load(path, map_location="cpu", weights_only=True)
    if not isinstance(obj, (tuple, list)) or len(obj) < 2:
        raise ValueError(f"{path}: expected a (data, slices) tuple, got {type(obj).__name__}")
    mapping, slices = _mapping_of(obj[0]), obj[1]
    if not isinstance(slices, dict):
        raise ValueError(f"{path}: slices must be a dict, got {type(slices).__name__}")
    return mapping, {k: torch.as_tensor(v) for k, v in slices.items()}


class CollatedDataset:
    """``InMemoryDataset`` surface over a (data, slices) pair: ``data`` (a :class:`Data` of the
    concatenated tensors), ``slices``, ``len()`` and ``[i]`` -> one molecule's :class:`Data`."""

    # the concatenation dimension of each key in PyG's collate (edge_index: -1, the rest 0)
    _CAT_DIM = {"edge_index": 1}

    def __init__(self, mapping: dict, slices: dict):
        self.data = Data(**mapping)
        self.slices = slices
        self._n = int(next(iter(slices.values())).numel()) - 1

    @classmethod
    def load(cls, path: str) -> "CollatedDataset":
        return cls(*load_collated(path))

    def __len__(self):
        return self._n

    def __getitem__(self, i: int) -> Data:
        if not -self._n <= i < self._n:
            raise IndexError(i)
        i %= self._n
        out = {}
        for k, v in self.data._store.items():
            if k not in self.slices:
                continue
            lo, hi = int(self.slices[k][i]), int(self.slices[k][i + 1])
            dim = self._CAT_DIM.get(k, 0)
            out[k] = v.narrow(dim, lo, hi - lo) if torch.is_tensor(v) and v.dim() > 0 else v
        d = Data(**out)
        if "edge_index" in out and "x" in out:
            ei = out["edge_index"]
            n = int(out["x"].shape[0])
            object.__setattr__(d, "_meta", {"nodes": np.array([n]), "edges": np.array([ei.shape[1]]),
                                            "triplets": np.array([triplet_count(ei.numpy(), n)])})
        if "edge_num" in out and torch.is_tensor(out["edge_num"]) and out["edge_num"].numel() == 1:
            d.edge_num = int(out["edge_num"].reshape(-1)[0])
        return d

    def atoms_per_molecule(self) -> torch.Tensor:
        return self.slices["x"][1:] - self.slices["x"][:-1]


def prepare_target(dataset: CollatedDataset, target: int, atom_ref: torch.Tensor | None = None) -> float:
    """train_ema.py:29-38 on ``dataset.data.y`` ([M, 12]) in place; returns ``print_calibration``."""
    ref = atom_reference_table() if atom_ref is None else atom_ref
    counts = dataset.atoms_per_molecule()
    owner = torch.arange(len(dataset)).repeat_interleave(counts)
    mol_ref = torch.zeros(len(dataset), dtype=ref.dtype).index_add_(0, owner, ref[target][dataset.data.x])
    y = dataset.data.y[:, target].squeeze() - mol_ref
    if target in EV_TARGETS:
        y = y * HARTREE_TO_EV
        calib = PRINT_CALIBRATION_EV
    else:
        calib = 1
    dataset.data.y = y
    return calib


def model_for_target(target: int, cfg: dict, device="cuda", pool_option="mean"):
    """train_ema.py:41-44: AtomWise ``xgnn_poly`` for targets 6-11, MolWise ``xgnn_poly_global``
    (``pool_option`` 'mean' or 'add') for 0-5."""
    from .xgnn import xgnn_poly, xgnn_poly_global
    if target in ATOMWISE_TARGETS:
        return xgnn_poly(device=device, **cfg)
    return xgnn_poly_global(device=device, pool_option=pool_option, **cfg)
