"""Oracle (test infrastructure): line-graph triplets, restating vertex_to_edge_2
(edge_graph.py:12-30).

For every directed edge e = (a -> b) in edge order and every k in N_out(b) in ascending order
with k != a, emit (src = id(b -> k), dst = e, j = b, i = a, k).  ``vertex_to_edge`` is the
vectorised numpy form; ``brute_force`` the literal double loop for small graphs.
"""
from __future__ import annotations

import numpy as np


def vertex_to_edge(edge_index: np.ndarray, num_nodes: int):
    """Returns (triplets [2,T] int64 (src; dst), atom_j, atom_i, atom_k)."""
    src, dst = np.asarray(edge_index[0], np.int64), np.asarray(edge_index[1], np.int64)
    E = src.shape[0]
    # edge ids grouped by source atom, destinations ascending (scipy CSR row order)
    order = np.lexsort((dst, src))
    rowptr = np.zeros(num_nodes + 1, np.int64)
    np.add.at(rowptr, src + 1, 1)
    rowptr = np.cumsum(rowptr)
    out_dst = dst[order]
    deg = rowptr[dst + 1] - rowptr[dst]            # |N_out(b)| for every e
    e_rep = np.repeat(np.arange(E), deg)            # destination line node, repeated
    start = np.repeat(rowptr[dst], deg)
    within = np.arange(deg.sum()) - np.repeat(np.cumsum(deg) - deg, deg)
    pos = start + within                            # CSR position of (b -> k)
    k = out_dst[pos]
    a = src[e_rep]
    keep = k != a
    e_rep, pos, k, a = e_rep[keep], pos[keep], k[keep], a[keep]
    trip = np.stack([order[pos], e_rep])
    return trip, dst[e_rep], a, k


def brute_force(edge_index, num_nodes):
    src, dst = [int(v) for v in edge_index[0]], [int(v) for v in edge_index[1]]
    eid = {(s, d): i for i, (s, d) in enumerate(zip(src, dst))}
    nbr = [[] for _ in range(num_nodes)]
    for s, d in zip(src, dst):
        nbr[s].append(d)
    rows = []
    for e, (a, b) in enumerate(zip(src, dst)):
        for k in sorted(nbr[b]):
            if k != a:
                rows.append((eid[(b, k)], e, b, a, k))
    if not rows:
        z = np.zeros(0, np.int64)
        return np.zeros((2, 0), np.int64), z, z, z
    r = np.array(rows, dtype=np.int64)
    return r[:, :2].T.copy(), r[:, 2], r[:, 3], r[:, 4]
