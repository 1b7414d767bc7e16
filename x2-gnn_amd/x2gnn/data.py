"""Minimal PyG-compatible ``Data`` / ``Batch`` (the operator surface the reference consumes).

The reference's ``xgnn_poly.forward(data)`` (xgnn.py:38-75) reads ``data.x`` (atomic numbers),
``data.edge_index`` (int64 [2,E], molecule-offset, sorted by source atom), ``data.edge_attr``
([E,338]), ``data.atom_pos`` ([N,3]), ``data.edge_num`` (directed edges per molecule),
``data.batch`` and ``data.num_graphs`` and tests ``"batch" in data._store`` (xgnn.py:41).  PyG
2.1's ``Batch.from_data_list`` collate increments ``edge_index`` by the running atom count and
stacks per-graph scalars; this module restates exactly that for the keys X2-GNN uses.

Besides the tensors, a collated batch carries host-side size metadata (atoms, edges and
triplets per molecule).  The device path takes every size from it, so a forward never reads a
size back from the GPU (the reference syncs on ``int(batch.max())`` and on the CPU triplet
round-trip, xgnn.py:52-53, model.py:190).
"""
from __future__ import annotations

import numpy as np
import torch

from .synth import triplet_count


class _Store(dict):
    pass


class Data:
    """Attribute bag with a ``_store`` mapping (PyG ``Data`` semantics for the used keys)."""

    def __init__(self, **kwargs):
        object.__setattr__(self, "_store", _Store())
        object.__setattr__(self, "_meta", None)
        for k, v in kwargs.items():
            if v is not None:
                self._store[k] = v

    def __getattr__(self, key):
        store = object.__getattribute__(self, "_store")
        if key in store:
            return store[key]
        raise AttributeError(key)

    def __setattr__(self, key, value):
        prop = getattr(type(self), key, None)
        if isinstance(prop, property):
            if prop.fset is not None:
                prop.fset(self, value)
            else:  # PyG stores into _store when the property has no setter
                self._store[key] = value
            return
        self._store[key] = value

    def __contains__(self, key):
        return key in self._store

    def keys(self):
        return list(self._store.keys())

    @property
    def num_nodes(self):
        return int(self._store["x"].shape[0])

    def to(self, device, non_blocking=False):
        out = type(self).__new__(type(self))
        object.__setattr__(out, "_store", _Store())
        object.__setattr__(out, "_meta", self._meta)
        for k, v in self._store.items():
            out._store[k] = v.to(device, non_blocking=non_blocking) if torch.is_tensor(v) else v
        return out

    def pin_memory(self):
        """A copy with every tensor in page-locked host memory (torch DataLoader(pin_memory=True) calls this), so
        ``to(device, non_blocking=True)`` overlaps the copy with device work."""
        out = type(self).__new__(type(self))
        object.__setattr__(out, "_store", _Store())
        object.__setattr__(out, "_meta", self._meta)
        for k, v in self._store.items():
            out._store[k] = v.pin_memory() if torch.is_tensor(v) else v
        return out

    def host_meta(self):
        """Per-molecule (atoms, edges, triplets) counts as int64 numpy arrays (host)."""
        if self._meta is None:
            object.__setattr__(self, "_meta", _meta_from_tensors(self))
        return self._meta


def _meta_from_tensors(data):
    """Host size metadata of a batch built without it (a Data made elsewhere, or a foreign PyG-style
    Batch): per-molecule atoms / edges / triplets, whether the directed edge set is symmetric, and the
    largest out-degree.  On the device (x2g_batch_meta: one pass over the edges, then ONE small
    device->host copy of the per-molecule vectors; the reference itself copies edge_index to the host,
    xgnn.py:52); a batch on the host is counted with numpy."""
    if data.edge_index.is_cuda:
        return _meta_on_device(data)
    ei = data.edge_index.detach().cpu().numpy()
    n = int(data.x.shape[0])
    if "ptr" in data._store:
        ptr = data.ptr.detach().cpu().numpy()
        nodes = np.diff(ptr)
    else:
        nodes = np.array([n])
    en = data.edge_num
    edges = (en.detach().cpu().numpy().reshape(-1) if torch.is_tensor(en)
             else np.array([en]).reshape(-1)).astype(np.int64)
    trips = []
    e0, a0 = 0, 0
    for m in range(len(nodes)):
        sub = ei[:, e0:e0 + edges[m]] - a0
        trips.append(triplet_count(sub, int(nodes[m])))
        e0 += edges[m]
        a0 += nodes[m]
    return {"nodes": nodes.astype(np.int64), "edges": edges, "triplets": np.array(trips, dtype=np.int64),
            "symmetric": _is_symmetric(ei, n), "max_degree": int(np.bincount(ei[0]).max()) if ei.shape[1] else 0}


def _meta_on_device(data):
    """x2g_batch_meta over a CUDA batch: the metadata dict of ``host_meta`` plus, under "index", the int32
    index forms GraphPlan reads (the ones collate makes on the host for x2gnn's own batches)."""
    from . import _lib
    from ._lib import call, ptr, stream_ptr

    ei = data.edge_index
    if ei.dtype != torch.int64:
        ei = ei.to(torch.int64)
    ei = ei.contiguous()
    dev = ei.device
    x = data.x.reshape(-1)
    x = (x if x.dtype == torch.int64 else x.to(torch.int64)).contiguous()
    E, n = int(ei.shape[1]), int(x.shape[0])
    st = data._store
    batch = st["batch"].to(torch.int64).contiguous() if "batch" in st else None
    B = int(data.num_graphs) if batch is not None else 1
    # every int32 output in one allocation (views), the host block in another
    buf = torch.empty(4 * E + 2 * n + 1 + 2 * (B + 1), dtype=torch.int32, device=dev)
    src, dst, src_t, dst_t, atom_t, rowptr, line_ptr, mol_ptr = torch.split(
        buf, [E, E, E, E, n, n + 1, B + 1, B + 1])
    info = torch.empty(3 * B + 6, dtype=torch.int64, device=dev)
    _lib.load()
    call("x2g_batch_meta", ptr(ei), ptr(x), ptr(batch), E, n, B, ptr(src), ptr(dst), ptr(src_t), ptr(dst_t),
         ptr(atom_t), ptr(line_ptr), ptr(mol_ptr), ptr(rowptr), ptr(info), stream_ptr())
    host = info.cpu().numpy()  # the one device->host copy: sizes per molecule and the flags
    # the center-atom kernels' schedule (degree order, the fused forward's packs and atom_info), made on the device
    # as collate makes it on the host for x2gnn's own batches (data.center_packs); enqueued after the read-back,
    # which then waits for nothing it does not need
    from .ops import center_schedule

    c_order, p_order, p_ptr, a_info = center_schedule(rowptr, src_t, n)
    mp_, lp, tr, fl = host[:B + 1], host[B + 1:2 * B + 2], host[2 * B + 2:3 * B + 2], host[3 * B + 2:]
    if fl[2]:
        raise ValueError("edge_index must list each directed edge once, sorted by (source, destination) "
                         "(the order the reference's radius graph emits, atom_graph.py:42-45)")
    index = {"_x2g_edge_src": src, "_x2g_edge_dst": dst, "_x2g_src_type": src_t, "_x2g_dst_type": dst_t,
             "_x2g_atom_type": atom_t, "_x2g_line_ptr": line_ptr, "_x2g_mol_ptr": mol_ptr,
             "_x2g_symmetric": bool(fl[0] == 0), "_x2g_max_degree": int(fl[1]),
             "_x2g_center_order": c_order, "_x2g_pack_order": p_order, "_x2g_center_packs": p_ptr,
             "_x2g_pack_info": a_info, "_x2g_center_rows": CENTER_SF_MAX_ROWS, "_x2g_center_mixed": True}
    if fl[3] == 0 and B > 0:  # every edge inside its molecule: the per-molecule line-graph builder
        index["_x2g_mol_trips"] = info[2 * B + 2:3 * B + 2]  # (a view of the device block: no copy)
        index["_x2g_max_mol_atoms"] = int(np.diff(mp_).max())
    return {"nodes": np.diff(mp_), "edges": np.diff(lp), "triplets": tr, "symmetric": bool(fl[0] == 0),
            "max_degree": int(fl[1]), "index": index}


class Batch(Data):
    """Collated molecules (PyG ``Batch.from_data_list`` restated for X2-GNN's keys)."""

    @property
    def num_graphs(self):
        return int(self._meta["nodes"].shape[0])

    @classmethod
    def from_data_list(cls, data_list):
        out = cls()
        nodes = np.array([d.num_nodes for d in data_list], dtype=np.int64)
        edges = np.array([int(d.edge_index.shape[1]) for d in data_list], dtype=np.int64)
        trips = []
        for d in data_list:
            if d._meta is not None:
                trips.append(int(d._meta["triplets"][0]))
            else:
                trips.append(triplet_count(d.edge_index.numpy(), d.num_nodes))
        object.__setattr__(out, "_meta", {"nodes": nodes, "edges": edges,
                                          "triplets": np.array(trips, dtype=np.int64)})
        offs = np.concatenate([[0], np.cumsum(nodes)[:-1]])
        keys = data_list[0].keys()
        for k in keys:
            vals = [d._store[k] for d in data_list]
            if k == "edge_index":
                out._store[k] = torch.cat([v + int(o) for v, o in zip(vals, offs)], dim=1)
            elif torch.is_tensor(vals[0]) and vals[0].dim() > 0:
                out._store[k] = torch.cat(vals, dim=0)
            else:
                out._store[k] = torch.as_tensor(np.array([np.asarray(v) for v in vals]).reshape(-1))
        out._store["batch"] = torch.from_numpy(np.repeat(np.arange(len(data_list), dtype=np.int64), nodes))
        out._store["ptr"] = torch.as_tensor(np.concatenate([[0], np.cumsum(nodes)]))
        _add_device_indices(out, nodes, edges)
        return out


def _add_device_indices(b, nodes, edges):
    """The int32 index forms the device path consumes (GraphPlan.from_atom_batch), made here on
    the host with the rest of the collate instead of by cast / cumsum / gather kernels in every
    step: edge source / destination atoms, the molecule atom and line-node offsets and each line
    node's destination element.  Under private ``_x2g_`` keys; a batch without them (built
    elsewhere) takes the device fallback."""
    ei = b._store.get("edge_index")
    if ei is None or "x" not in b._store:
        return
    ei_np = ei.numpy()
    b._store["_x2g_edge_src"] = torch.from_numpy(np.ascontiguousarray(ei_np[0], dtype=np.int32))
    b._store["_x2g_edge_dst"] = torch.from_numpy(np.ascontiguousarray(ei_np[1], dtype=np.int32))
    b._store["_x2g_mol_ptr"] = torch.from_numpy(np.concatenate([[0], np.cumsum(nodes)]).astype(np.int32))
    b._store["_x2g_line_ptr"] = torch.from_numpy(np.concatenate([[0], np.cumsum(edges)]).astype(np.int32))
    b._store["_x2g_dst_type"] = torch.from_numpy(b._store["x"].numpy()[ei_np[1]].astype(np.int32))
    b._store["_x2g_src_type"] = torch.from_numpy(b._store["x"].numpy()[ei_np[0]].astype(np.int32))
    b._store["_x2g_atom_type"] = torch.from_numpy(b._store["x"].numpy().reshape(-1).astype(np.int32))
    b._store["_x2g_symmetric"] = _is_symmetric(ei_np, int(nodes.sum()))
    # per-molecule triplet counts for the per-molecule line-graph builder (x2g_vertex_to_edge_sym_mol); the
    # molecules' edges stay inside them by construction (each collated from its own graph)
    trips = b._meta.get("triplets") if b._meta is not None else None
    if trips is not None and len(trips) == len(nodes):
        b._store["_x2g_mol_trips"] = torch.from_numpy(np.ascontiguousarray(trips, dtype=np.int64))
        b._store["_x2g_max_mol_atoms"] = int(nodes.max()) if len(nodes) else 0
    deg = np.bincount(ei_np[0], minlength=int(nodes.sum()))
    b._store["_x2g_max_degree"] = int(deg.max()) if deg.size else 0
    if not HOST_SCHEDULE:  # the plan makes it on the device (ops.center_schedule) from the built line graph
        b._store["_x2g_device_schedule"] = True
        return
    # the center-atom kernels' workgroups: one atom each by decreasing degree (the longest blocks first), and
    # the fused forward's units of atoms packed by degree (the longest units first)
    b._store["_x2g_center_order"] = torch.from_numpy(np.argsort(-deg, kind="stable").astype(np.int32))
    order, packs, rows = center_packs(deg)
    b._store["_x2g_pack_order"] = torch.from_numpy(order)
    b._store["_x2g_center_packs"] = torch.from_numpy(packs)
    # the leading units of more rows than the fused forward's LDS image holds (single atoms: the source-tiled
    # kernel), and the largest row count of the rest
    hubs, rows = center_hubs(deg, order, packs)
    b._store["_x2g_center_hubs"] = hubs
    b._store["_x2g_center_rows"] = rows
    # per pack-order position: (atom, first out-edge, degree, element): the fused forward's row tables in one
    # load per atom (x2g_sbf_attention_fwd_center_sf atom_info)
    first = np.concatenate([[0], np.cumsum(deg)[:-1]]) if deg.size else deg
    z = b._store["x"].numpy().reshape(-1)
    info = np.stack([order, first[order], deg[order], z[order]], axis=1).astype(np.int32)
    b._store["_x2g_pack_info"] = torch.from_numpy(np.ascontiguousarray(info).reshape(-1))


# The center kernels' schedule (degree order, the fused forward's packs, atom_info) of a collated batch: made
# here on the host (center_packs: best fit over the whole batch) or, False, on the device when the step builds
# the batch's line graph (ops.center_schedule: best fit per window of 64 atoms), which takes it off the collate.
HOST_SCHEDULE = True

CENTER_PACK_ROWS = 16  # the center kernels' half-wave owners per workgroup (csrc/attention_center.hip)
CENTER_PACK_MEMBERS = 16


def center_packs(deg, cap=CENTER_PACK_ROWS, max_members=CENTER_PACK_MEMBERS):
    """Workgroup units of the center-atom attention kernels (x2g_sbf_attention_fwd_center_sf / _bwd_center
    pack_ptr): the atoms packed best-fit-decreasing by degree into units of at most ``cap`` rows (a unit's
    rows are its atoms' out-edges; one workgroup's 16 half-wave owners take one row each), an atom of
    degree >= cap alone, atoms without edges ``max_members`` to a unit.  One atom per workgroup keeps only
    57 % of the owners busy at config 2 (degrees 2-17); these units keep 90 %.  Returns (order int32 [N]:
    the atoms unit by unit, packs int32 [P + 1]: unit p = order[packs[p] .. packs[p + 1]), max_rows: the
    largest unit's row count), the units in decreasing order of their largest degree (the longest
    workgroups start first)."""
    import ctypes

    from . import _lib

    deg = np.ascontiguousarray(deg, dtype=np.int64)
    n = int(deg.shape[0])
    order = np.empty(n, dtype=np.int32)
    packs = np.empty(n + 1, dtype=np.int32)
    units, rows = ctypes.c_int64(0), ctypes.c_int32(0)
    # the best fit is a sequential loop over the atoms: native (csrc/line_graph.hip), a Python loop took two
    # thirds of a 128-molecule collate (tests/test_host.py checks it against that loop)
    _lib.call("x2g_center_packs_host", deg.ctypes.data, n, int(cap), int(max_members), order.ctypes.data,
              packs.ctypes.data, ctypes.addressof(units), ctypes.addressof(rows))
    return order, packs[:units.value + 1].copy(), int(rows.value)


CENTER_SF_MAX_ROWS = 17  # ops.CENTER_SF_MAX_ROWS


def center_hubs(deg, order, packs, max_rows=CENTER_SF_MAX_ROWS):
    """(hubs, rows): the units of center_packs' (order, packs) are by decreasing largest degree, so those of
    more than ``max_rows`` rows (single atoms) are the first ``hubs``; ``rows`` is the largest row count of
    the others."""
    deg = np.asarray(deg, dtype=np.int64)
    if len(packs) < 2:
        return 0, 0
    urows = np.add.reduceat(deg[order], packs[:-1]) if len(order) else np.zeros(len(packs) - 1, np.int64)
    big = urows > max_rows
    hubs = int(np.argmin(big)) if not big.all() else int(len(big))
    assert not big[hubs:].any(), "units over the row bound must lead"
    return hubs, int(urows[hubs:].max(initial=0))


def _is_symmetric(ei, n):
    """True when the directed edge set contains b->a for every a->b (checked exactly, host side)."""
    if ei.shape[1] == 0:
        return True
    fwd = ei[0].astype(np.int64) * n + ei[1]
    rev = ei[1].astype(np.int64) * n + ei[0]
    sf = np.sort(fwd)
    # duplicate directed edges break the symmetric builders' per-edge counts (deg(b) - 1): such a
    # multigraph takes the generic path even when its multiset is symmetric
    if sf.size > 1 and bool((sf[1:] == sf[:-1]).any()):
        return False
    return bool(np.array_equal(sf, np.sort(rev)))


def molecule_to_data(mol: dict) -> Data:
    """One synthetic/xyz molecule dict (see :mod:`x2gnn.synth`) as a ``Data``."""
    d = Data(
        x=torch.as_tensor(mol["x"], dtype=torch.int64),
        atom_pos=torch.as_tensor(mol["atom_pos"], dtype=torch.float32),
        edge_index=torch.as_tensor(mol["edge_index"], dtype=torch.int64),
        edge_attr=torch.as_tensor(mol["edge_attr"], dtype=torch.float32) if "edge_attr" in mol else None,
        edge_num=int(mol["edge_num"]),
        y=float(mol.get("y", 0.0)),
    )
    object.__setattr__(d, "_meta", {"nodes": np.array([len(mol["x"])]),
                                    "edges": np.array([int(mol["edge_num"])]),
                                    "triplets": np.array([int(mol["triplet_num"])])})
    return d


def collate(mols) -> Batch:
    """Molecule dicts -> collated ``Batch`` on the host: Batch.from_data_list([molecule_to_data(m) ...]) (PyG's
    collate restated, with y as float32) computed straight from the dicts' arrays — one numpy concatenation
    per key instead of a Data object and five tensors per molecule (tests/test_host.py checks the two equal)."""
    B = len(mols)
    nodes = np.fromiter((len(m["x"]) for m in mols), dtype=np.int64, count=B)
    edges = np.fromiter((int(m["edge_num"]) for m in mols), dtype=np.int64, count=B)
    trips = np.fromiter((int(m["triplet_num"]) for m in mols), dtype=np.int64, count=B)
    offs = np.concatenate([[0], np.cumsum(nodes)[:-1]])
    b = Batch()
    object.__setattr__(b, "_meta", {"nodes": nodes, "edges": edges, "triplets": trips})
    st = b._store
    st["x"] = torch.from_numpy(np.concatenate([np.asarray(m["x"], dtype=np.int64).reshape(-1) for m in mols]))
    st["atom_pos"] = torch.from_numpy(np.concatenate([np.asarray(m["atom_pos"], dtype=np.float32).reshape(-1, 3)
                                                      for m in mols]))
    st["edge_index"] = torch.from_numpy(np.concatenate(
        [np.asarray(m["edge_index"], dtype=np.int64).reshape(2, -1) + o for m, o in zip(mols, offs)], axis=1))
    if "edge_attr" in mols[0]:
        st["edge_attr"] = torch.from_numpy(np.concatenate([np.asarray(m["edge_attr"], dtype=np.float32)
                                                           for m in mols]))
    st["edge_num"] = torch.from_numpy(edges.copy())
    st["y"] = torch.from_numpy(np.array([float(m.get("y", 0.0)) for m in mols], dtype=np.float32))
    # np.repeat: torch.repeat_interleave took 0.2-7 ms of a 128-molecule collate, after the edge_attr copy
    st["batch"] = torch.from_numpy(np.repeat(np.arange(B, dtype=np.int64), nodes))
    st["ptr"] = torch.from_numpy(np.concatenate([[0], np.cumsum(nodes)]))
    _add_device_indices(b, nodes, edges)
    return b
