"""Write tests/golden/pyg_inmemory_v21.pt (+ .npz with the expected tensors).

The reference's processed dataset (qm9_allprop.py:58) is ``torch.save(InMemoryDataset.collate
(datas))`` under torch_geometric 2.1.0 — a pickled ``(Data, slices)`` whose Data object names
``torch_geometric.data.data.Data`` / ``DataTensorAttr`` / ``DataEdgeAttr`` and
``torch_geometric.data.storage.GlobalStorage``.  PyG is not installed here and the reference
ships no processed file, so this script builds a file with the same pickle structure from
stand-in classes registered under those module paths (PyG 2.1.0's ``Data.__init__`` fills
``_tensor_attr_cls``, ``_edge_attr_cls`` and ``_store``; ``BaseStorage.__getstate__`` pickles
``_mapping`` and the dereferenced ``_parent``), collated the way PyG's ``collate(increment=
False)`` does for the qm9_allprop keys.  Parity of the reader against a real PyG file is
therefore unpinned; this pins the layout as restated.

    python tests/golden/make_pyg_fixture.py
"""
from __future__ import annotations

import os
import sys
import types
import weakref
from dataclasses import dataclass

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "x2-gnn_amd"))

from x2gnn.synth import radius_edges, random_geometry  # noqa: E402


def _install_fake_pyg():
    pkg = types.ModuleType("torch_geometric")
    data_pkg = types.ModuleType("torch_geometric.data")
    data_mod = types.ModuleType("torch_geometric.data.data")
    storage_mod = types.ModuleType("torch_geometric.data.storage")

    @dataclass
    class DataTensorAttr:
        attr_name: str = None
        index: object = None

    @dataclass
    class DataEdgeAttr:
        layout: object = None
        is_sorted: bool = False
        size: tuple = None

    class GlobalStorage:
        def __init__(self, _parent=None):
            self.__dict__["_mapping"] = {}
            self.__dict__["_parent"] = weakref.ref(_parent)

        def __getstate__(self):
            out = self.__dict__.copy()
            out["_parent"] = out["_parent"]()
            return out

    class Data:
        def __init__(self, **kwargs):
            self.__dict__["_tensor_attr_cls"] = DataTensorAttr
            self.__dict__["_edge_attr_cls"] = DataEdgeAttr
            self.__dict__["_store"] = GlobalStorage(_parent=self)
            for k, v in kwargs.items():
                self._store._mapping[k] = v

    for cls, mod in ((DataTensorAttr, data_mod), (DataEdgeAttr, data_mod), (Data, data_mod),
                     (GlobalStorage, storage_mod)):
        cls.__module__ = mod.__name__
        cls.__qualname__ = cls.__name__
        setattr(mod, cls.__name__, cls)
    for m in (pkg, data_pkg, data_mod, storage_mod):
        sys.modules[m.__name__] = m
    return Data


def main():
    Data = _install_fake_pyg()
    rng = np.random.default_rng(77)
    mols = []
    for m in range(3):
        z, pos = random_geometry(rng, 1.8, n_heavy=3 + m, n_h=3)
        pos = pos.astype(np.float32)
        ei = radius_edges(pos.astype(np.float64), 5.0)
        ea = (0.1 * rng.standard_normal((ei.shape[1], 338))).astype(np.float32)
        y = rng.standard_normal((1, 12)).astype(np.float32)
        mols.append(dict(x=torch.from_numpy(z), edge_index=torch.from_numpy(ei), edge_attr=torch.from_numpy(ea),
                         y=torch.from_numpy(y), edge_num=torch.tensor([ei.shape[1]]), idx=torch.tensor([m]),
                         atom_pos=torch.from_numpy(pos)))
    keys = ["x", "edge_index", "edge_attr", "y", "edge_num", "idx", "atom_pos"]
    cat, slices = {}, {}
    for k in keys:
        dim = 1 if k == "edge_index" else 0
        vals = [mm[k] for mm in mols]
        cat[k] = torch.cat(vals, dim=dim)
        sizes = torch.tensor([v.shape[dim] for v in vals])
        slices[k] = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(sizes, 0)])
    torch.save((Data(**cat), slices), os.path.join(HERE, "pyg_inmemory_v21.pt"))
    exp = {f"{k}_{i}": mm[k].numpy() for i, mm in enumerate(mols) for k in keys}
    exp.update({f"slices_{k}": v.numpy() for k, v in slices.items()})
    np.savez_compressed(os.path.join(HERE, "pyg_inmemory_v21.npz"), n=np.int64(len(mols)), **exp)
    print("wrote", len(mols), "molecules")


if __name__ == "__main__":
    main()
