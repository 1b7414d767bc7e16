"""Per-batch device plan: every index structure the hot path needs, built once per forward.

The reference recomputes these implicitly inside each operator (scatter sizes via
``int(batch.max()) + 1`` host syncs at model.py:190 and inside PyG's LayerNorm/softmax, the
triplets via a CPU round trip at xgnn.py:52-53).  Here they are built once on the device from
host-side size metadata, so a whole forward+backward enqueues without a single device->host
read (and can be captured in a HIP graph).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import ops
from .data import _meta_from_tensors


class GraphPlan:
    """Index structures of one collated batch.

    lg            LineGraph (triplets, CSR by destination; source-major transpose on demand)
    atom_rowptr   [N+1]  line nodes (= directed edges) grouped by source atom, i.e. the CSR of
                         ``edge_index_0`` that AtomWise pools over (readout.py:37)
    line_ptr      [B+1]  line nodes per molecule (graph LayerNorm segments, model.py:183)
    mol_ptr       [B+1]  atoms per molecule (global add pool, model.py:190)
    dst_type      [E]    atomic number of the middle atom b of each line node e=(a->b): the
                         row of the per-element edge table every triplet into e uses
    num_atoms, num_lines, num_triplets, num_graphs, out_graphs (host ints)
    """

    def __init__(self):
        self.lg = None
        self.atom_rowptr = self.line_ptr = self.mol_ptr = self.dst_type = None
        self.num_atoms = self.num_lines = self.num_triplets = self.num_graphs = self.out_graphs = 0
        # int32 [1] device flags of the index contracts checked without a host read (from_line_data)
        self.order_status = []

    def order_violated(self) -> bool:
        """True when an index this plan assumed sorted was not (reads the device flags: one sync;
        call it where a check is wanted, e.g. in tests or after a run)."""
        return any(bool(s.item()) for s in self.order_status)

    # ------------------------------------------------------------------ from an atom batch
    @classmethod
    def from_atom_batch(cls, data):
        """Plan for ``xgnn_poly.forward(data)`` inputs (edge_index sorted by (src, dst)).

        ``data`` is x2gnn's collated Batch (host size metadata and the int32 index forms ride
        along) or any PyG-style batch exposing the keys xgnn.py:38-75 reads (``_store``, ``x``,
        ``edge_index``, ``edge_num``, ``ptr`` / ``batch``): for a foreign batch the per-molecule
        sizes are derived from its tensors here (one device->host copy of edge_index, as the
        reference's own CPU triplet builder makes, xgnn.py:52-53)."""
        host_meta = getattr(data, "host_meta", None)
        meta = host_meta() if callable(host_meta) else _meta_from_tensors(data)
        p = cls()
        nodes, edges, trips = meta["nodes"], meta["edges"], meta["triplets"]
        p.num_atoms, p.num_lines, p.num_triplets = int(nodes.sum()), int(edges.sum()), int(trips.sum())
        p.num_graphs = int(len(nodes))
        nz = np.nonzero(edges)[0]
        # the reference sizes the pool by the last molecule that has line nodes (model.py:190)
        p.out_graphs = int(nz[-1]) + 1 if len(nz) else 0
        ei = data.edge_index
        dev = ei.device
        # the int32 index forms: collate's (x2gnn's own batches) or x2g_batch_meta's (a foreign batch)
        st = meta.get("index") or data._store
        within = False  # every edge known to stay inside its molecule (collate's batches; x2g_batch_meta flag 3)
        if "_x2g_edge_src" in st and st["_x2g_edge_src"].device == dev:
            mols = None
            if st.get("_x2g_mol_trips") is not None and st["_x2g_mol_trips"].device == dev:
                mols = (st["_x2g_mol_ptr"], st["_x2g_line_ptr"], st["_x2g_mol_trips"], st["_x2g_max_mol_atoms"])
                within = True
            p.lg = ops.LineGraph(st["_x2g_edge_src"], st["_x2g_edge_dst"], p.num_atoms, p.num_triplets,
                                 st.get("_x2g_symmetric", False), molecules=mols)
            p.line_ptr, p.mol_ptr, p.dst_type = st["_x2g_line_ptr"], st["_x2g_mol_ptr"], st["_x2g_dst_type"]
            src_type = st.get("_x2g_src_type")
            p.lg.atom_type = st.get("_x2g_atom_type")
            p.lg.center_order = st.get("_x2g_center_order")
            p.lg.pack_order = st.get("_x2g_pack_order")
            p.lg.center_packs = st.get("_x2g_center_packs")
            p.lg.center_rows = st.get("_x2g_center_rows")
            p.lg.pack_info = st.get("_x2g_pack_info")
            p.lg.center_hubs = st.get("_x2g_center_hubs", 0)
            p.lg.center_mixed = st.get("_x2g_center_mixed", False)
            if st.get("_x2g_device_schedule", False) and p.lg.edge_rev is not None:  # (data.HOST_SCHEDULE False)
                sched = ops.center_schedule(p.lg.atom_rowptr, src_type, p.num_atoms)
                p.lg.center_order, p.lg.pack_order, p.lg.center_packs, p.lg.pack_info = sched
                p.lg.center_rows, p.lg.center_mixed = ops.CENTER_SF_MAX_ROWS, True
        else:
            p.lg = ops.vertex_to_edge(ei, p.num_atoms, p.num_triplets, meta.get("symmetric", False))
            p.line_ptr = _ptr_from_counts(data.edge_num, p.num_graphs, dev)
            if "ptr" in st:
                p.mol_ptr = ops._i32(data.ptr)
            else:
                p.mol_ptr = (torch.arange(2, device=dev, dtype=torch.int32) * p.num_atoms)
            p.dst_type = ops._i32(data.x.index_select(0, p.lg.edge_dst))
            src_type = None
        if src_type is None:
            src_type = ops._i32(data.x.index_select(0, p.lg.edge_src.long()))
        if p.lg.atom_type is None:
            p.lg.atom_type = ops._i32(data.x.reshape(-1))
        p.lg.dst_type, p.lg.src_type = p.dst_type, src_type
        p.atom_rowptr = p.lg.atom_rowptr
        # per-molecule line-node / triplet counts on the host: whole-molecule ranges of the triplet
        # stream for the tiled inference attention (ops._infer_tiles), with no device read; the atoms
        # per molecule only when no edge joins two molecules (the tiled center forward assumes a tile's
        # atoms own exactly its triplets: otherwise the destination-major tiles)
        p.lg.mol_counts = (np.asarray(edges, dtype=np.int64), np.asarray(trips, dtype=np.int64)) + (
            (np.asarray(nodes, dtype=np.int64),) if within else ())
        # the largest center-atom degree (host metadata): sizes the center-atom kernels' LDS image
        md = st.get("_x2g_max_degree", meta.get("max_degree"))
        p.lg.max_degree = int(md) if md is not None else None
        return p

    # ------------------------------------------------------------------ from line-graph tensors
    @classmethod
    def from_line_data(cls, data, edge_index_0, atom_batch):
        """Plan for the drop-in ``SBFTransformer.forward(data, edge_index_0, atom_batch)`` API.

        The molecule count is read back from the device (``int(batch.max()) + 1``, as the reference
        does at model.py:53 and inside PyG's LayerNorm); nothing else is.  The four index vectors
        must be sorted ascending, as the reference produces them (vertex_to_edge_2 emits triplets
        by destination; PyG batches are ordered by molecule; edge_index is source-sorted): their row
        pointers come from ``ops.csr_rowptr_checked``, which flags a violation on the device.  In an
        eager call the flags come back with the molecule count (the same host read) and an unsorted
        index raises ValueError instead of giving wrong sums; under HIP-graph capture nothing is
        read and ``order_violated()`` reports it after a replay.  The fast path through ``xgnn_poly``
        never takes this branch.
        """
        p = cls()
        p.num_lines = int(data.x.shape[0])
        p.num_atoms = int(atom_batch.shape[0])
        p.num_triplets = int(data.edge_index.shape[1])
        p.lg = ops.LineGraph.from_triplets(data.edge_index, p.num_lines)
        p.atom_rowptr, st_a = ops.csr_rowptr_checked(edge_index_0, p.num_atoms)
        b = data.batch
        p.num_graphs = p.out_graphs = int(b.max()) + 1 if b.numel() else 0
        p.line_ptr, st_l = ops.csr_rowptr_checked(b, p.num_graphs)
        p.mol_ptr, st_m = ops.csr_rowptr_checked(atom_batch, p.num_graphs)
        p.order_status = [p.lg.order_status, st_a, st_l, st_m]
        if not torch.cuda.is_current_stream_capturing():
            bad = torch.cat(p.order_status).cpu().tolist()
            names = ("data.edge_index[1] (triplet destinations)", "edge_index_0", "data.batch", "atom_batch")
            wrong = [n for n, f in zip(names, bad) if f]
            if wrong:
                raise ValueError("SBFTransformer drop-in: index not sorted ascending (or out of range): "
                                 + ", ".join(wrong))
        return p


def _ptr_from_counts(counts, n, device):
    if torch.is_tensor(counts):
        c = counts.reshape(-1).to(device=device)
    else:
        c = torch.full((1,), int(counts), device=device, dtype=torch.int64)
    return F.pad(torch.cumsum(c, 0), (1, 0)).to(torch.int32)

