"""Device operators of the hot path: thin wrappers over libx2g.so + their autograd rules.

Every function here runs on the GPU through the C ABI (include/x2g.h) on PyTorch's current
stream; inputs must be CUDA (HIP) tensors.  There is deliberately no CPU fallback.

Operator                     replaces (reference / un-vendored dependency)
---------------------------  ----------------------------------------------------------------
``vertex_to_edge``           edge_graph.vertex_to_edge_2 (edge_graph.py:12-30), scipy on CPU
``bessel_env`` /             F_B_2D.forward (angular_basis_layer.py:80-93) + poly_envelop
``spherical_basis``          (envelop.py:16-21) + the angle code of xgnn.py:61-65
``sbf_attention``            SBFTransformerConv.propagate/message/softmax/aggregate + skip
                             (sbftransformer_conv.py:99-162; PyG MessagePassing, utils.softmax)
``segment_sum``              torch_scatter.scatter_add with a sorted index (readout.py:37,
                             model.py:190) and its backward gather
``segment_softmax``          torch_geometric.utils.softmax
``graph_layer_norm``         torch_geometric.nn.LayerNorm(mode='graph') (model.py:161,183)
"""
from __future__ import annotations

import contextlib
import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

EDGE_NONE, EDGE_PER_TRIPLET, EDGE_PER_DST = 0, 1, 2


def rows_fit(rows, width):
    """True when a [rows, width] fp32 array is addressable by the kernels' 32-bit BYTE offsets
    (buffer-resource loads / stores: num_records is a byte count below 2^31)."""
    return int(rows) * int(width) * 4 < 2 ** 31


def _need_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("x2gnn device ops need GPU tensors (no CPU fallback by design)")


def _f32(t):
    return t if t.dtype == torch.float32 and t.is_contiguous() else t.to(torch.float32).contiguous()


def _i32(t):
    return t if t.dtype == torch.int32 and t.is_contiguous() else t.to(torch.int32).contiguous()


# ---------------------------------------------------------------------------------- line graph
MOL_ROWPTR_MAX_ATOMS = 16384  # x2g_vertex_to_edge_sym_mol's per-molecule degree histogram (64 KB of LDS)


class LineGraph:
    """Triplet structure of one collated batch (all int32, on the device).

    trip_rowptr/trip_src/trip_dst: CSR by destination line node, in the reference's order.
    atom_i/atom_j/atom_k: the three atoms of each triplet (xgnn.py:52 edge_i/edge_j/edge_k).
    src_rowptr/src_perm: the same triplets grouped by source line node (built on first use).
    """

    def __init__(self, edge_src, edge_dst, num_nodes, num_triplets, symmetric=False, with_transpose=None,
                 molecules=None):
        """``with_transpose`` (default: symmetric and grad enabled, i.e. a backward will ask for
        ``src_csr``): build the by-source lists with the line graph (x2g_line_graph_sym_build,
        three launches for both instead of five).  ``molecules`` = (mol_ptr int32 [B+1], line_ptr int32
        [B+1], triplets per molecule int64 [B], largest molecule's atom count) of a symmetric batch whose
        edges stay inside their molecules: the row pointers one workgroup per molecule
        (x2g_vertex_to_edge_sym_mol, two launches), the transpose left to ``src_csr`` (the center-atom
        backward never reads it)."""
        self.symmetric = bool(symmetric)  # caller-asserted: b->a present for every a->b (x2g_*_sym)
        if molecules is not None and (not self.symmetric or int(molecules[3]) > MOL_ROWPTR_MAX_ATOMS
                                      or int(molecules[2].shape[0]) < 1):
            molecules = None
        if with_transpose is None:
            with_transpose = self.symmetric and torch.is_grad_enabled() and molecules is None
        self.E = int(edge_src.shape[0])
        self.N = int(num_nodes)
        self.T = int(num_triplets)
        self.edge_src, self.edge_dst = edge_src, edge_dst
        dev = edge_src.device
        i32 = dict(dtype=torch.int32, device=dev)
        self.atom_rowptr = torch.empty(self.N + 1, **i32)
        self.trip_rowptr = torch.empty(self.E + 1, **i32)
        self.trip_src = torch.empty(self.T, **i32)
        self.trip_dst = torch.empty(self.T, **i32)
        self.atom_j = torch.empty(self.T, **i32)
        self.atom_i = torch.empty(self.T, **i32)
        self.atom_k = torch.empty(self.T, **i32)
        self._src_rowptr = None
        self._src_perm = None
        self._src_dst = None
        self.order_status = None  # built here in order: nothing to check
        # per-line-node element rows of the x2g_vertex_to_edge line graph (GraphPlan sets them):
        # dst_type[e] = Z of e's destination atom = the edge row of every triplet into e, and
        # src_type[s] = Z of s's source atom = the same row for every triplet out of s
        self.dst_type = self.src_type = None
        ws_bytes = int(_lib.load().x2g_vertex_to_edge_workspace(self.E, self.N))
        self._ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        # symmetric graphs: each edge's reverse and where its triplet block starts, for the center-atom
        # attention kernels (written by the same emission grid)
        self.edge_rev = torch.empty(self.E, **i32) if self.symmetric else None
        self.rev_trip = torch.empty(self.E, **i32) if self.symmetric else None
        # degree bound of the center atoms (host metadata; set by GraphPlan, None = unknown) and each atom's
        # element row (int32 [N]: the key of the center-atom edge-term gradient)
        self.max_degree = None
        self.atom_type = None
        # the center kernels' workgroups (collate's; None: the identity): int32 [N] the atoms by decreasing
        # degree (one per workgroup), and the fused forward's packs (data.center_packs): int32 [N] the atoms
        # unit by unit, int32 [P + 1] the units' bounds in it, the largest row count of the units after the
        # first center_hubs (single atoms of more rows than the fused forward's LDS image holds: the tiled form)
        self.center_order = self.pack_order = self.center_packs = self.center_rows = self.pack_info = None
        self.center_hubs = 0
        self.center_mixed = False  # the schedule is x2g_center_schedule's (hub units among the packs)
        if molecules is not None:
            mol_ptr, line_ptr, trips, max_atoms = molecules
            call("x2g_vertex_to_edge_sym_mol", ptr(edge_src), ptr(edge_dst), self.E, self.N, self.T, ptr(mol_ptr),
                 ptr(line_ptr), ptr(trips), int(trips.shape[0]), int(max_atoms), ptr(self.atom_rowptr),
                 ptr(self.trip_rowptr), ptr(self.trip_src), ptr(self.trip_dst), ptr(self.atom_j), ptr(self.atom_i),
                 ptr(self.atom_k), ptr(self.edge_rev), ptr(self.rev_trip), stream_ptr())
            return
        if with_transpose and self.symmetric:
            self._src_rowptr = torch.empty(self.E + 1, **i32)
            self._src_perm = torch.empty(self.T, **i32)
            self._src_dst = torch.empty(self.T, **i32)
            call("x2g_line_graph_sym_build", ptr(edge_src), ptr(edge_dst), self.E, self.N, self.T,
                 ptr(self.atom_rowptr), ptr(self.trip_rowptr), ptr(self.trip_src), ptr(self.trip_dst),
                 ptr(self.atom_j), ptr(self.atom_i), ptr(self.atom_k), ptr(self._src_rowptr), ptr(self._src_perm),
                 ptr(self._src_dst), ptr(self.edge_rev), ptr(self.rev_trip), ptr(self._ws), ws_bytes, stream_ptr())
            return
        if self.symmetric:
            call("x2g_vertex_to_edge_sym", ptr(edge_src), ptr(edge_dst), self.E, self.N, self.T, ptr(self.atom_rowptr),
                 ptr(self.trip_rowptr), ptr(self.trip_src), ptr(self.trip_dst), ptr(self.atom_j), ptr(self.atom_i),
                 ptr(self.atom_k), ptr(self.edge_rev), ptr(self.rev_trip), ptr(self._ws), ws_bytes, stream_ptr())
            return
        call("x2g_vertex_to_edge", ptr(edge_src), ptr(edge_dst), self.E, self.N, self.T, ptr(self.atom_rowptr),
             ptr(self.trip_rowptr), ptr(self.trip_src), ptr(self.trip_dst), ptr(self.atom_j), ptr(self.atom_i),
             ptr(self.atom_k), ptr(self._ws), ws_bytes, stream_ptr())

    @classmethod
    def from_triplets(cls, triplet_index, num_line_nodes: int):
        """Wrap an existing triplet index [2, T] whose row 1 is sorted ascending (as vertex_to_edge_2
        emits it).  Nothing is read back: the order is checked on the device and a violation is
        flagged in ``order_status`` (int32 [1]; see ``order_violated``), the row pointer staying in
        range either way."""
        lg = cls.__new__(cls)
        lg.E, lg.N, lg.T = int(num_line_nodes), None, int(triplet_index.shape[1])
        lg.edge_src = lg.edge_dst = lg.atom_rowptr = None
        lg.atom_i = lg.atom_j = lg.atom_k = None
        lg.trip_src = _i32(triplet_index[0])
        lg.trip_dst = _i32(triplet_index[1])
        lg.trip_rowptr, lg.order_status = csr_rowptr_checked(lg.trip_dst, lg.E)
        lg._src_rowptr = lg._src_perm = lg._src_dst = None
        lg.dst_type = lg.src_type = None
        lg.symmetric = False
        lg.edge_rev = lg.rev_trip = lg.max_degree = lg.atom_type = None
        lg.center_order = lg.pack_order = lg.center_packs = lg.center_rows = lg.pack_info = None
        lg.center_hubs = 0
        lg.center_mixed = False
        ws_bytes = int(_lib.load().x2g_vertex_to_edge_workspace(lg.E, 0))
        lg._ws = torch.empty(ws_bytes, dtype=torch.uint8, device=lg.trip_src.device)
        return lg

    def src_csr(self):
        """(src_rowptr [E+1], src_perm [T]): the triplets grouped by source line node; ``src_dst``
        [T] (each source-major position's destination) is built with them."""
        if self._src_rowptr is None:
            dev = self.trip_src.device
            self._src_rowptr = torch.empty(self.E + 1, dtype=torch.int32, device=dev)
            self._src_perm = torch.empty(self.T, dtype=torch.int32, device=dev)
            self._src_dst = torch.empty(self.T, dtype=torch.int32, device=dev)
            if self.symmetric:  # lists written in order from the degrees (no atomics, no segment sort)
                call("x2g_line_graph_transpose_sym", ptr(self.edge_src), ptr(self.edge_dst), ptr(self.atom_rowptr),
                     ptr(self.trip_rowptr), self.E, ptr(self._src_rowptr), ptr(self._src_perm), ptr(self._src_dst),
                     ptr(self._ws), self._ws.numel(), stream_ptr())
            else:
                call("x2g_line_graph_transpose", ptr(self.trip_src), ptr(self.trip_dst), self.T, self.E,
                     ptr(self._src_rowptr), ptr(self._src_perm), ptr(self._src_dst), ptr(self._ws),
                     self._ws.numel(), stream_ptr())
        return self._src_rowptr, self._src_perm

    @property
    def src_dst(self):
        self.src_csr()
        return self._src_dst

    def order_violated(self) -> bool:
        """True when the triplet destinations handed to ``from_triplets`` were not sorted (one sync)."""
        return self.order_status is not None and bool(self.order_status.item())

    def triplet_index(self):
        """int64 [2, T] (row 0 = source line node id(b->k), row 1 = destination id(a->b))."""
        return torch.stack([self.trip_src.long(), self.trip_dst.long()])


def vertex_to_edge(edge_index, num_nodes: int, num_triplets: int, symmetric: bool = False) -> LineGraph:
    """Build the line graph of a (src, dst)-sorted directed edge list on the device
    (``symmetric``: the caller asserts b->a exists for every a->b)."""
    _need_cuda(edge_index)
    ei = _i32(edge_index)
    return LineGraph(ei[0].contiguous(), ei[1].contiguous(), num_nodes, num_triplets, symmetric)


def csr_rowptr(sorted_keys, num_segments: int):
    _need_cuda(sorted_keys)
    keys = _i32(sorted_keys)
    out = torch.empty(num_segments + 1, dtype=torch.int32, device=keys.device)
    call("x2g_csr_rowptr", ptr(keys), keys.numel(), num_segments, ptr(out), stream_ptr())
    return out


def csr_rowptr_checked(keys, num_segments: int):
    """(rowptr [num_segments + 1], status int32 [1]) for keys assumed sorted and in range: no host
    read; status is 1 on the device when the assumption fails (x2g_csr_rowptr_checked)."""
    _need_cuda(keys)
    k = _i32(keys.reshape(-1))
    out = torch.empty(num_segments + 1, dtype=torch.int32, device=k.device)
    status = torch.empty(1, dtype=torch.int32, device=k.device)
    call("x2g_csr_rowptr_checked", ptr(k), k.numel(), num_segments, ptr(out), ptr(status), stream_ptr())
    return out, status


# ---------------------------------------------------------------------------------- basis
def bessel_env(dist, cutoff: float = 5.0, num_spherical: int = 7, num_radial: int = 6):
    """[E] distances -> [E, num_spherical * num_radial] env(d) * N_ln j_l(z_ln d / cutoff)."""
    _need_cuda(dist)
    d = _f32(dist)
    out = torch.empty(d.shape[0], num_spherical * num_radial, dtype=torch.float32, device=d.device)
    call("x2g_bessel_env", ptr(d), d.shape[0], float(cutoff), num_spherical, num_radial, ptr(out), stream_ptr())
    return out


class _EdgeBasis(torch.autograd.Function):
    """dist, env, rbf_env = sin(freq * d / cutoff) * env, bessel_env in one kernel
    (x2g_edge_basis); the backward gives the RadialBasis.frequencies gradient."""

    @staticmethod
    def forward(ctx, freq, pos, lg, cutoff, nsph, nrad):
        E, R = lg.E, freq.shape[0]
        f32 = dict(dtype=torch.float32, device=pos.device)
        dist, env = torch.empty(E, **f32), torch.empty(E, **f32)
        rbf, bes = torch.empty(E, R, **f32), torch.empty(E, nsph * nrad, **f32)
        call("x2g_edge_basis", ptr(_f32(pos)), ptr(lg.edge_src), ptr(lg.edge_dst), E, float(cutoff), ptr(_f32(freq)), R,
             nsph, nrad, ptr(dist), ptr(env), ptr(rbf), ptr(bes), stream_ptr())
        ctx.save_for_backward(dist, env, freq)
        ctx.freq_param = freq  # the Parameter object itself (grad_sink looks at its attributes)
        ctx.cutoff = float(cutoff)
        ctx.mark_non_differentiable(dist, env, bes)
        ctx.set_materialize_grads(False)
        return dist, env, rbf, bes

    @staticmethod
    def backward(ctx, _gd, _ge, grbf, _gb):
        if grbf is None or not ctx.needs_input_grad[0]:
            return None, None, None, None, None, None
        dist, env, freq = ctx.saved_tensors
        E, R = dist.shape[0], freq.shape[0]
        lib = _lib.load()
        sink = grad_sink(ctx.freq_param)
        dfreq = sink if sink is not None else torch.empty(R, dtype=torch.float32, device=dist.device)
        ws_bytes = int(lib.x2g_edge_basis_freq_grad_workspace(E, R))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dist.device)
        defer = sink is not None and _defer() is not None and E > 0
        flags = (ACCUM_WGRAD if sink is not None else 0) | (DEFER_SLAB_SUM if defer else 0)
        call("x2g_edge_basis_freq_grad", ptr(_f32(grbf)), ptr(dist), ptr(env), ptr(freq), E, R, ctx.cutoff, ptr(dfreq),
             flags, ptr(ws), ws_bytes, stream_ptr())
        if defer:
            _defer_job(ws, 0, int(lib.x2g_edge_basis_freq_grad_splits(E)), R, 0, dfreq, None)
        return (None if sink is not None else dfreq), None, None, None, None, None


def edge_basis(pos, lg: LineGraph, freq, cutoff: float = 5.0, num_spherical: int = 7, num_radial: int = 6):
    """(dist [E], env [E], rbf_env [E, R] = sin(freq d / cutoff) env, bessel_env [E, num_spherical *
    num_radial]) for the line graph's directed edges; rbf_env carries the gradient to ``freq``
    (xgnn.py:49-53,66-70)."""
    _need_cuda(pos, freq)
    return _EdgeBasis.apply(freq, pos, lg, cutoff, int(num_spherical), int(num_radial))


def spherical_basis(pos, lg: LineGraph, rbf_env, want_cos=False, num_spherical: int = 7, num_radial: int = 6,
                    lazy=False):
    """[T, S] sbf = rbf_env[src] * Y_l0(theta) (S = num_spherical * num_radial, l-major), theta from
    the triplet's atom positions.

    When gradients are being recorded the two factors are kept on the line graph
    (``lg.sbf_factors = (sbf, rbf_env, Y[T, 8])``): the attention backward then folds lin_sbf's
    weight gradient per source line node instead of materialising d(lin_sbf(sbf)) [T, D]
    (csrc/attention_fold.inc)."""
    _need_cuda(pos, rbf_env)
    pos = _f32(pos)
    rbf_env = _f32(rbf_env)
    S = num_spherical * num_radial
    out = torch.empty(lg.T, S, dtype=torch.float32, device=pos.device)
    cos_t = torch.empty(lg.T, dtype=torch.float32, device=pos.device) if want_cos else None
    # the factors are kept for the factorised backward and for the fused-projection center forward (which
    # also runs without grad, in inference: its source-tiled form takes every degree up to the center kernels'
    # bound)
    sf_fits = getattr(lg, "max_degree", None) is not None and lg.max_degree <= CENTER_MAX_DEGREE
    fold = _FOLD_SBF and (num_spherical, num_radial) == FOLD_BASIS and (torch.is_grad_enabled() or sf_fits)
    ylm = torch.empty(lg.T, 8, dtype=torch.float32, device=pos.device) if fold else None
    # lazy (the model's own forward): only the factors are written; the [T, S] rows are filled by
    # materialize_sbf when a consumer reads them (the fused center forward never does: 586 MB per step at
    # config 5, 33 MB at config 2)
    lazy = lazy and fold and not want_cos
    call("x2g_spherical_basis", ptr(pos), ptr(lg.atom_i), ptr(lg.atom_j), ptr(lg.atom_k), None, ptr(lg.trip_src),
         ptr(rbf_env), lg.T, num_spherical, num_radial, None if lazy else ptr(out), ptr(cos_t), ptr(ylm),
         stream_ptr())
    lg.sbf_factors = (out, rbf_env, ylm) if ylm is not None else None
    lg.sbf_pending = (out, pos, rbf_env, num_spherical, num_radial) if lazy else None
    return (out, cos_t) if want_cos else out


# The model's own forward asks spherical_basis for the factors only (lazy sbf rows): False = always write
# the [T, S] rows (a constant: bench.py --no-lazy-sbf and the parity tests flip it).
LAZY_SBF = True


def materialize_sbf(lg, sbf):
    """Fill the [T, S] sbf rows a lazy spherical_basis left unwritten, if ``sbf`` is them (every consumer that
    reads sbf values, rather than its factors, calls this first)."""
    pend = getattr(lg, "sbf_pending", None)
    if pend is None or pend[0] is not sbf:
        return sbf
    out, pos, rbf_env, ns, nr = pend
    call("x2g_spherical_basis", ptr(pos), ptr(lg.atom_i), ptr(lg.atom_j), ptr(lg.atom_k), None, ptr(lg.trip_src),
         ptr(rbf_env), lg.T, ns, nr, ptr(out), None, None, stream_ptr())
    lg.sbf_pending = None
    return sbf


def spherical_basis_from_angles(theta, trip_src, rbf_env, num_spherical: int = 7, num_radial: int = 6):
    """[T, S] sbf = rbf_env[trip_src] * Y_l0(theta) for given angles (F_B_2D signature)."""
    _need_cuda(theta, trip_src, rbf_env)
    th = _f32(theta)
    src = _i32(trip_src)
    out = torch.empty(th.shape[0], num_spherical * num_radial, dtype=torch.float32, device=th.device)
    call("x2g_spherical_basis", None, None, None, None, ptr(th), ptr(src), ptr(_f32(rbf_env)), th.shape[0],
         num_spherical, num_radial, ptr(out), None, None, stream_ptr())
    return out


# ---------------------------------------------------------------------------------- attention
# Graph LayerNorm after the conv (model.py:46) fused: the attention forward leaves per-row (mean, M2)
# statistics (x2g_sbf_attention_fwd_stats) and the trunk's row chain normalises its input while
# staging it (x2g_chain_fwd_ln) instead of a LayerNorm pass over the rows.  False: separate.
#
# The module switches below (_LN_FUSE, _LN_BWD_ROWS, _SRC_G, _FOLD_SBF, _DEFER_KEYED, INFER_TILE,
# _CHAIN, _FAN_IN, _POOL_BATCH) are constants, not environment reads: each exists because a parity
# test flips it to check the fused path against the plain one (tests/test_gpu_model.py,
# tests/test_gpu_kernels.py).  Paths that were measured slower and had no such test are deleted.
_LN_FUSE = True
# With the fused LayerNorm, its backward's per-molecule sums come from per-row sums the chain
# backward leaves (x2g_chain_bwd_ln + x2g_graph_layernorm_bwd_rows): False = the two-pass LN backward.
_LN_BWD_ROWS = True
# The folded source-major pass recomputes g_t = d loss / d a_t (per head) itself — bitwise the value
# the destination pass computes — so g [T, H] is neither written nor read: False = the round trip.
_SRC_G = True

# Factorised lin_sbf backward (csrc/attention_fold.inc): False restores the two-pass backward +
# [T, D] d_sbfproj + T-row weight GEMM (the drop-in conv API takes it anyway: its sbf is an
# arbitrary [T, 42] tensor).
_FOLD_SBF = True
FOLD_BASIS = (7, 6)  # the (num_spherical, num_radial) the folded kernels are compiled for (sbf_dim 42)


def _sbf_factors(lg, sbf, edge_mode, D, edge, edge_row):
    fac = getattr(lg, "sbf_factors", None)
    if (fac is None or fac[0] is not sbf or edge_mode == EDGE_PER_TRIPLET or D not in (32, 64, 128)
            or sbf.shape[1] != FOLD_BASIS[0] * FOLD_BASIS[1]):
        return None
    if edge_mode == EDGE_PER_DST and (edge_row is None or edge is None or edge.shape[0] > 16):
        return None  # the source pass stages the per-destination edge table in LDS
    return fac[1], fac[2]


CENTER_MAX_DEGREE = 128  # X2G_CENTER_MAX_DEGREE
# Center-atom attention kernels (csrc/attention_center.hip) for symmetric line graphs: False = the
# destination-major kernels everywhere; _CENTER_BWD False = the center forward with the destination-major
# backward passes (parity tests flip them).
_CENTER = True
_CENTER_BWD = True
# The center forward with lin_sbf fused (x2g_sbf_attention_fwd_center_sf: S_t rebuilt from the sbf factors
# per center atom, no projection launch, no S read; S rows stored only for a backward): False = project S
# first and read it (x2g_sbf_project + x2g_sbf_attention_fwd_center).
_CENTER_SF = True


def _center_units(lg, packed):
    """(order, pack_ptr or None, units, max_rows, atom_info or None) of a whole-batch center kernel: with
    ``packed`` the batch's packs of atoms (data.center_packs) when it has them, else one atom per
    workgroup by decreasing degree."""
    packs = getattr(lg, "center_packs", None)
    if packed and packs is not None and lg.pack_order is not None and lg.center_rows is not None:
        return lg.pack_order, packs, int(packs.shape[0]) - 1, max(int(lg.center_rows), 1), \
            getattr(lg, "pack_info", None)
    return lg.center_order, None, lg.N, max(int(lg.max_degree), 1), None


# Units of more rows than this go to the source-tiled fused forward (x2g_sbf_attention_fwd_center_sf_tiled):
# the fused forward's LDS image of 17 rows (81.7 KB) is the largest that keeps two workgroups per CU
# (data.CENTER_SF_MAX_ROWS; config 2's largest degree is 17, config 5's AID atoms reach 61).
CENTER_SF_MAX_ROWS = 17


def _center_split(lg):
    """(order, pack_ptr, info, launches): the fused forward's units and the launches that cover them, each
    (entry, unit0, n_units, rows, skip_rows): with collate's packs the first ``center_hubs`` units (single
    atoms of more than CENTER_SF_MAX_ROWS rows, by decreasing degree) take the source-tiled form and the rest
    (at most ``center_rows`` rows each) the untiled one; with a device-made schedule (x2g_center_schedule:
    hubs among the packs) both forms run over all units, each leaving out the other's (skip_rows / max_rows);
    without either (unpacked) every atom is a unit by decreasing degree, all of them tiled when any exceeds
    the bound."""
    order, packs, units, rows, info = _center_units(lg, _PACK_FWD)
    sf, tiled = "x2g_sbf_attention_fwd_center_sf", "x2g_sbf_attention_fwd_center_sf_tiled"
    if packs is not None and getattr(lg, "center_mixed", False):
        launches = [(sf, 0, units, CENTER_SF_MAX_ROWS, 0)]
        if lg.max_degree > CENTER_SF_MAX_ROWS:
            launches.insert(0, (tiled, 0, units, lg.max_degree, CENTER_SF_MAX_ROWS))
        return order, packs, info, launches
    if packs is not None:
        hubs = int(getattr(lg, "center_hubs", 0) or 0)
        launches = [(tiled, 0, hubs, lg.max_degree, 0)] if hubs else []
        if units > hubs:
            launches.append((sf, hubs, units - hubs, rows, 0))
        return order, packs, info, launches
    if rows > CENTER_SF_MAX_ROWS:
        return order, None, None, [(tiled, 0, units, lg.max_degree, 0)]
    return order, None, None, [(sf, 0, units, rows, 0)]


def center_schedule(atom_rowptr, src_row, num_atoms: int):
    """The center kernels' schedule made on the device (x2g_center_schedule): (center_order [N], pack_order [N],
    pack_ptr [N + 1], atom_info [N * 4]) — the same kind data.center_packs makes on the host (best fit per
    window of 64 atoms, the units by decreasing largest degree); its hub units lead the packs, which the
    launches find on the device (LineGraph.center_mixed)."""
    n = int(num_atoms)
    dev = atom_rowptr.device
    off = 4 * ((3 * n + 1 + 3) // 4)  # atom_info 16-byte aligned after the order / pack order / pack_ptr
    buf = torch.empty(off + 4 * n, dtype=torch.int32, device=dev)
    c_order, p_order, p_ptr = torch.split(buf[:3 * n + 1], [n, n, n + 1])
    info = buf[off:off + 4 * n]
    lib = _lib.load()
    ws_b = int(lib.x2g_center_schedule_workspace(n))
    ws = torch.empty(ws_b, dtype=torch.uint8, device=dev)
    call("x2g_center_schedule", ptr(atom_rowptr), ptr(src_row), n, ptr(c_order), ptr(p_order), ptr(p_ptr),
         ptr(info), ptr(ws), ws_b, stream_ptr())
    return c_order, p_order, p_ptr, info


def _center_launch(launches, common, outs):
    for entry, u0, n, rows, skip in launches:
        if entry.endswith("_tiled"):
            call(entry, *common, u0, n, rows, skip, *outs)
        else:
            call(entry, *common, u0, n, rows, *outs)


# Workgroup packs (data.center_packs) in the fused forward: 16 owners per workgroup keep 90 % instead of
# 57 % of them busy, and its owners never wait for one another (no barrier after the P products).  The
# backward stays one atom per workgroup on 4 waves: with packs (8 waves) its phase barriers waited for
# the longest member's owners and it measured 4 % slower (profiles/r5k_*); the packed backward was removed.
_PACK_FWD = True
# The fused forward hands the center backward each source's P rows (E x 3.5 KB) instead of every S row
# (T x 512 B), and the backward rebuilds S_t = b + sum_l Y_l(t) P_s[l] bit for bit: False = S rows.
_CENTER_P = True


def _unit_rows_lds(rows):  # csrc/attention_center.hip unit_rows_lds
    return ((3 * rows + 2 * 32 + 4) * 4 + 15) // 16 * 16


def _center_sf_ok(lg, factors, D):
    """Whether the fused-projection center forward applies: the sbf factors are this call's (the units of more
    rows than its LDS image holds take its source-tiled form)."""
    if not (_CENTER_SF and factors is not None and factors[1] is not None and D == 128 and lg.max_degree is not None):
        return False
    _, _, _, launches = _center_split(lg)
    return all(e.endswith("_tiled") or _unit_rows_lds(r) + 4776 * r <= 160 * 1024 for e, _, _, r, _ in launches)


def _center_bwd_ok(lg, heads, s_rows=False):
    """Whether the center-atom backward takes this line graph (its element rows known, the LDS image of the
    largest atom's block within 160 KB, and its T-row arrays within the kernel's 32-bit buffer offsets:
    the S rows T x 512 B when ``s_rows``, else the P-row form's (g, a) scratch T x heads x 8 B)."""
    row_bytes = 128 * 4 if s_rows else heads * 8
    return (_CENTER_BWD and getattr(lg, "atom_type", None) is not None and lg.max_degree is not None and
            lg.T * row_bytes < 2 ** 31 and
            _lib.load().x2g_sbf_attention_bwd_center_lds(lg.max_degree, heads) <= 160 * 1024)


def _center_rows(lg, edge_mode, edge_row, D, channels):
    """(ok, src_row): whether the center-atom forward applies to this call, and the per-source edge-table
    row it reads for EDGE_PER_DST (the center atom's element: lg.src_type, valid when the caller's
    per-destination rows are the line graph's own dst_type)."""
    if (not _CENTER or getattr(lg, "edge_rev", None) is None or lg.max_degree is None
            or lg.max_degree > CENTER_MAX_DEGREE or D != 128 or channels % 4 or edge_mode == EDGE_PER_TRIPLET):
        return False, None
    if edge_mode == EDGE_PER_DST:
        if edge_row is None or lg.src_type is None or edge_row is not lg.dst_type:
            return False, None
        return True, lg.src_type
    return True, None


class _SBFAttention(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, skip, edge, sbf, w_sbf, b_sbf, lg, edge_mode, edge_row, heads, channels,
                keep_alpha=True):
        w_param, b_param = w_sbf, b_sbf
        # its gradient is read only by the table chain's backward, which flushes deferred sums first
        pending = getattr(edge, "_x2g_keyed_pending", None)
        ctx.defer_edge = _DEFER_KEYED and pending is not None and ctx.needs_input_grad[4]
        ctx.keyed_pending = pending
        factors = _sbf_factors(lg, sbf, edge_mode, heads * channels, edge, edge_row)
        q, k, v, skip = _f32(q), _f32(k), _f32(v), _f32(skip)
        sbf, w_sbf, b_sbf = _f32(sbf), _f32(w_sbf), _f32(b_sbf)
        edge = _f32(edge) if edge is not None else None
        E, T, D = q.shape[0], lg.T, heads * channels
        dev = q.device
        out = torch.empty(E, D, dtype=torch.float32, device=dev)
        center, src_row = _center_rows(lg, edge_mode, edge_row, D, channels)
        # the P-row center backward (the shipped training path) recomputes the logits from rows it stages
        p_bwd = center and _CENTER_P and _center_sf_ok(lg, factors, D) and _center_bwd_ok(lg, heads)
        # the logits [T, H] are read by the other backwards or for the attention weights; the center forwards
        # skip the store otherwise (inference: 223 MB per layer at config 5; training: 12 MB written and read
        # back per layer at config 2)
        alpha = (torch.empty(T, heads, dtype=torch.float32, device=dev)
                 if keep_alpha or not center or (_keeps(ctx) and not p_bwd) else None)
        smax = torch.empty(E, heads, dtype=torch.float32, device=dev)
        sden = torch.empty(E, heads, dtype=torch.float32, device=dev)
        # per-row (mean, M2) of the output for a graph LayerNorm fused into the next row chain
        rstats = torch.empty(E, 2, dtype=torch.float32, device=dev) if _LN_FUSE and D == 128 else None
        sbf_p = None
        if center and _center_sf_ok(lg, factors, D):
            # lin_sbf fused into the center forward: S_t rebuilt per center atom from the sbf factors; for a
            # backward, the sources' P rows (the center backward rebuilds S_t from them) or the S rows
            sproj = None
            if _keeps(ctx):
                if p_bwd:
                    sbf_p = torch.empty(E, 7, D, dtype=torch.float32, device=dev)
                else:
                    sproj = torch.empty(T, D, dtype=torch.float32, device=dev)
            # (the atoms beyond the untiled form's LDS image take the source-tiled form: _center_split)
            order, packs, info, launches = _center_split(lg)
            common = (ptr(q), ptr(k), ptr(v), ptr(skip), ptr(edge), ptr(src_row), edge_mode, ptr(factors[0]),
                      ptr(factors[1]), ptr(w_sbf), ptr(b_sbf), ptr(lg.atom_rowptr), ptr(lg.edge_rev),
                      ptr(lg.rev_trip), ptr(order), ptr(packs), ptr(info))
            outs = (E, T, heads, channels, ptr(out), ptr(alpha), ptr(smax), ptr(sden), ptr(rstats), ptr(sproj),
                    ptr(sbf_p), stream_ptr())
            _center_launch(launches, common, outs)
        else:
            # S = lin_sbf(sbf) once per layer [T, D], right before this layer's attention (so it is still
            # in the MALL when the attention kernels read its rows: sbf pointer = S, weight pointer NULL)
            # instead of re-projecting per triplet
            sproj = torch.empty(T, D, dtype=torch.float32, device=dev)
            materialize_sbf(lg, sbf)
            call("x2g_sbf_project", ptr(sbf), T, sbf.shape[1], ptr(w_sbf), ptr(b_sbf), D, ptr(sproj), stream_ptr())
            if center:
                call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(edge), ptr(src_row),
                     edge_mode, ptr(sproj), 0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip),
                     ptr(lg.center_order), 0, lg.N, lg.max_degree, E, T, heads, channels, ptr(out), ptr(alpha),
                     ptr(smax), ptr(sden), ptr(rstats), stream_ptr())
            else:
                call("x2g_sbf_attention_fwd_stats" if rstats is not None else "x2g_sbf_attention_fwd", ptr(q),
                     ptr(k), ptr(v), ptr(skip), ptr(edge), ptr(edge_row), edge_mode, ptr(sproj), None, None,
                     ptr(lg.trip_rowptr), ptr(lg.trip_src), E, T, heads, channels, D, ptr(out), ptr(alpha),
                     ptr(smax), ptr(sden), *((ptr(rstats),) if rstats is not None else ()), stream_ptr())
        if factors is not None:  # the factorised backward never reads sbf itself
            ctx.save_for_backward(q, k, v, edge, factors[0], factors[1], sproj, alpha, smax, sden, sbf_p,
                                  b_sbf if sbf_p is not None else None)
        else:
            ctx.save_for_backward(q, k, v, edge, sbf, None, sproj, alpha, smax, sden, None, None)
        ctx.fold = factors is not None
        ctx.w_param, ctx.b_param = w_param, b_param
        ctx.lg, ctx.edge_mode, ctx.edge_row, ctx.heads, ctx.channels = lg, edge_mode, edge_row, heads, channels
        ctx.edge_shape = None if edge is None else edge.shape
        # (one call: a second mark_non_differentiable replaces the first's set)
        ctx.mark_non_differentiable(*(t for t in (alpha, smax, sden, rstats) if t is not None))
        # the logits / max / denominator outputs never receive gradients: do not let autograd
        # materialise zero-filled [T, H] / [E, H] tensors for them (three fill launches per layer)
        ctx.set_materialize_grads(False)
        return out, alpha, smax, sden, rstats

    @staticmethod
    def backward(ctx, dout, _da=None, _dm=None, _ds=None, _dr=None):
        q, k, v, edge, sbf, ylm, sproj, alpha, smax, sden, sbf_p, b_sbf = ctx.saved_tensors
        lg, mode, heads, channels = ctx.lg, ctx.edge_mode, ctx.heads, ctx.channels
        dout = _f32(dout)
        E, T, D = q.shape[0], lg.T, heads * channels
        dev = q.device
        dq = torch.empty(E, D, dtype=torch.float32, device=dev)
        dk = torch.empty_like(dq)
        dv = torch.empty_like(dq)
        if ctx.fold:  # sbf here is the radial factor rbf_env [E, 42]
            return _SBFAttention._backward_fold(ctx, dout, q, k, v, edge, sbf, ylm, sproj, alpha, smax, sden, dq, dk, dv,
                                                sbf_p, b_sbf)
        dlogit = torch.empty(T, heads, dtype=torch.float32, device=dev)
        dproj = torch.empty(T, D, dtype=torch.float32, device=dev)
        if mode == EDGE_PER_TRIPLET:
            d_edge = torch.empty(T, D, dtype=torch.float32, device=dev)
        elif mode == EDGE_PER_DST:
            d_edge = torch.empty(E, D, dtype=torch.float32, device=dev)
        else:
            d_edge = None
        st = stream_ptr()
        call("x2g_sbf_attention_bwd_dst", ptr(q), ptr(k), ptr(v), ptr(edge), ptr(ctx.edge_row), mode, ptr(sproj),
             None, None, ptr(lg.trip_rowptr), ptr(lg.trip_src), ptr(alpha), ptr(smax), ptr(sden), ptr(dout), E, T,
             heads, channels, D, ptr(dq), ptr(d_edge), ptr(dlogit), ptr(dproj), st)
        src_rowptr, src_perm = lg.src_csr()
        call("x2g_sbf_attention_bwd_src", ptr(q), ptr(sproj), None, None, ptr(src_rowptr), ptr(src_perm),
             ptr(lg.trip_dst), ptr(alpha), ptr(smax), ptr(sden), ptr(dlogit), ptr(dout), E, T, heads, channels, D,
             ptr(dk), ptr(dv), st)
        if not ctx.needs_input_grad[4]:
            d_edge = None
        elif mode == EDGE_PER_DST and ctx.edge_row is not None:
            # rows of the edge table are shared by many destinations: sum d_edge per table row
            d_edge = keyed_row_sum(d_edge, ctx.edge_row, ctx.edge_shape[0])
        gw, gb = grad_sink(ctx.w_param), grad_sink(ctx.b_param)
        materialize_sbf(lg, sbf)
        if gw is not None and gb is not None:
            dw, db = linear_wgrad(dproj, sbf, dw_out=gw, db_out=gb)  # summed into the bucket: None
        else:
            dw, db = linear_wgrad(dproj, sbf)
        return dq, dk, dv, dout, d_edge, None, dw, db, None, None, None, None, None, None

    @staticmethod
    def _backward_fold(ctx, dout, q, k, v, edge, radial, ylm, sproj, alpha, smax, sden, dq, dk, dv, sbf_p=None,
                       b_sbf=None):
        lg, mode, heads, channels = ctx.lg, ctx.edge_mode, ctx.heads, ctx.channels
        E, T, D = q.shape[0], lg.T, heads * channels
        dev = q.device
        # g[T, H] (d loss / d a_t): the source pass recomputes it from rows it holds anyway (_SRC_G)
        g = None if _SRC_G else torch.empty(T, heads, dtype=torch.float32, device=dev)
        prob = torch.empty(T, heads, dtype=torch.float32, device=dev)
        rho = torch.empty(E, heads, dtype=torch.float32, device=dev)
        gfold = torch.empty(E, 8, D, dtype=torch.float32, device=dev)
        st = stream_ptr()
        center, src_row = _center_rows(lg, mode, ctx.edge_row, D, channels)
        if sbf_p is not None or (center and _center_bwd_ok(lg, heads, s_rows=True)):
            # one launch for both passes, per center atom (csrc/attention_center.hip); the edge term's
            # gradient comes per center atom and is summed by the atoms' elements
            want_edge = mode == EDGE_PER_DST and ctx.needs_input_grad[4]
            d_edge_atom = torch.empty(lg.N, D, dtype=torch.float32, device=dev) if want_edge else None
            g_work = torch.empty(2, T, heads, dtype=torch.float32, device=dev)
            call("x2g_sbf_attention_bwd_center", ptr(q), ptr(k), ptr(v), ptr(edge), ptr(src_row), mode, ptr(sproj),
                 ptr(sbf_p), ptr(b_sbf), ptr(ylm), ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(lg.center_order),
                 ptr(alpha), ptr(smax), ptr(sden), ptr(dout), lg.N, lg.max_degree, E, T, heads, channels, ptr(dq),
                 ptr(dk), ptr(dv), ptr(gfold), ptr(d_edge_atom), ptr(g_work), st)
            d_edge = None
            if want_edge:
                if ctx.defer_edge:
                    d_edge = keyed_row_sum_deferred(d_edge_atom, lg.atom_type, ctx.edge_shape[0], ctx.keyed_pending)
                else:
                    d_edge = keyed_row_sum(d_edge_atom, lg.atom_type, ctx.edge_shape[0])
            gw, gb = grad_sink(ctx.w_param), grad_sink(ctx.b_param)
            if gw is not None and gb is not None:
                dw, db = sbf_radial_wgrad(gfold, radial, dw_out=gw, db_out=gb)
            else:
                dw, db = sbf_radial_wgrad(gfold, radial)
            return dq, dk, dv, dout, d_edge, None, dw, db, None, None, None, None, None, None
        d_edge = torch.empty(E, D, dtype=torch.float32, device=dev) if mode == EDGE_PER_DST else None
        call("x2g_sbf_attention_bwd_dst_g", ptr(q), ptr(k), ptr(v), ptr(edge), ptr(ctx.edge_row), mode, ptr(sproj),
             ptr(lg.trip_rowptr), ptr(lg.trip_src), ptr(alpha), ptr(smax), ptr(sden), ptr(dout), E, T, heads, channels,
             ptr(dq), ptr(d_edge), ptr(g), ptr(prob), ptr(rho), st)
        src_rowptr, src_perm = lg.src_csr()
        rows = 0 if edge is None else edge.shape[0]
        # the edge row per SOURCE (constant over a source segment) when the rows are the line graph's
        # own destination elements
        src_row = lg.src_type if (ctx.edge_row is not None and ctx.edge_row is lg.dst_type) else None
        call("x2g_sbf_attention_bwd_src_fold", ptr(q), ptr(v), ptr(edge), ptr(ctx.edge_row), ptr(src_row), rows, mode,
             ptr(sproj), ptr(ylm), ptr(src_rowptr), ptr(src_perm), ptr(lg.src_dst), ptr(lg.trip_dst), ptr(prob),
             ptr(g), ptr(rho), ptr(dout), E, T, heads, channels, ptr(dk), ptr(dv), ptr(gfold), st)
        if not ctx.needs_input_grad[4]:
            d_edge = None  # (written by the kernel; no consumer: the table's gradient is not wanted)
        elif mode == EDGE_PER_DST and ctx.edge_row is not None:
            if ctx.defer_edge:
                d_edge = keyed_row_sum_deferred(d_edge, ctx.edge_row, ctx.edge_shape[0], ctx.keyed_pending)
            else:
                d_edge = keyed_row_sum(d_edge, ctx.edge_row, ctx.edge_shape[0])
        gw, gb = grad_sink(ctx.w_param), grad_sink(ctx.b_param)
        if gw is not None and gb is not None:
            dw, db = sbf_radial_wgrad(gfold, radial, dw_out=gw, db_out=gb)
        else:
            dw, db = sbf_radial_wgrad(gfold, radial)
        return dq, dk, dv, dout, d_edge, None, dw, db, None, None, None, None, None, None


def sbf_radial_wgrad(gfold, radial, dw_out=None, db_out=None):
    """(dW_sbf [D, 42], db_sbf [D]) from the source-folded gradient G [E, 8, D] and the radial
    factor rbf_env [E, 42] (x2g_sbf_radial_wgrad); accumulates into dw_out/db_out when given."""
    E, _, D = gfold.shape
    accum = dw_out is not None
    if accum and db_out is None:
        raise ValueError("accumulating dW_sbf needs the bias-gradient buffer too")
    dw = dw_out if accum else torch.empty(D, 42, dtype=torch.float32, device=gfold.device)
    db = db_out if accum else torch.empty(D, dtype=torch.float32, device=gfold.device)
    lib = _lib.load()
    ws_bytes = int(lib.x2g_sbf_radial_wgrad_workspace(E, D))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=gfold.device)
    defer = accum and _defer() is not None and E > 0
    flags = (ACCUM_WGRAD if accum else 0) | (DEFER_SLAB_SUM if defer else 0)
    call("x2g_sbf_radial_wgrad", ptr(gfold), ptr(_f32(radial)), E, D, ptr(dw), ptr(db), flags, ptr(ws), ws_bytes,
         stream_ptr())
    if defer:
        _defer_job(ws, 0, int(lib.x2g_sbf_radial_wgrad_splits(E)), D * 42, D, dw, db)
    return (None, None) if accum else (dw, db)


class _EmbeddingTable(torch.autograd.Function):
    """Embedding rows per element with torch.embedding_renorm_ (in place) and the
    scale_grad_by_freq / padding_idx gradient rules, one launch each way (csrc/embedding.hip)."""

    @staticmethod
    def forward(ctx, weight, z, max_norm, padding_idx, scale_grad):
        V, D = weight.shape
        if weight.dtype != torch.float32 or not weight.is_contiguous():
            raise ValueError("embedding weight must be contiguous fp32")
        zz = z if z.dtype == torch.int64 and z.is_contiguous() else z.to(torch.int64).contiguous()
        table = torch.empty_like(weight)
        counts = torch.empty(V, dtype=torch.float32, device=weight.device)
        call("x2g_embedding_table", ptr(weight), ptr(zz), zz.numel(), V, D, float(max_norm or 0.0), ptr(counts),
             ptr(table), stream_ptr())
        ctx.save_for_backward(counts)
        ctx.w_param, ctx.pad, ctx.scale = weight, (-1 if padding_idx is None else int(padding_idx)), bool(scale_grad)
        return table

    @staticmethod
    def backward(ctx, g):
        (counts,) = ctx.saved_tensors
        V, D = counts.shape[0], g.shape[1]
        sink = grad_sink(ctx.w_param)
        dw = sink if sink is not None else torch.empty(V, D, dtype=torch.float32, device=g.device)
        call("x2g_embedding_table_bwd", ptr(_f32(g)), ptr(counts) if ctx.scale else None, V, D, ctx.pad, ptr(dw),
             ACCUM_WGRAD if sink is not None else 0, stream_ptr())
        return (None if sink is not None else dw), None, None, None, None


def embedding_table(weight, z, max_norm, padding_idx, scale_grad_by_freq):
    """Rows of ``weight`` per element (see _EmbeddingTable); renormalises the used rows in place."""
    _need_cuda(weight, z)
    return _EmbeddingTable.apply(weight, z, max_norm, padding_idx, scale_grad_by_freq)


class DenseFwdGroup(ctypes.Structure):
    _fields_ = [("x", ctypes.c_void_p), ("w", ctypes.c_void_p), ("b", ctypes.c_void_p), ("res", ctypes.c_void_p),
                ("y", ctypes.c_void_p), ("z", ctypes.c_void_p)]


class DenseBwdGroup(ctypes.Structure):
    _fields_ = [("dy", ctypes.c_void_p), ("z", ctypes.c_void_p), ("x", ctypes.c_void_p), ("w", ctypes.c_void_p),
                ("dx", ctypes.c_void_p), ("dx_add", ctypes.c_void_p), ("dw", ctypes.c_void_p),
                ("db", ctypes.c_void_p)]


class HeadGroup(ctypes.Structure):
    _fields_ = [("h", ctypes.c_void_p), ("w", ctypes.c_void_p), ("b", ctypes.c_void_p), ("dh", ctypes.c_void_p),
                ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p)]


def _dp(t):
    return t.data_ptr() if t is not None else None


def _wgrad_targets(params, shapes, dev):
    """Per parameter: (buffer, accum) — the bucket view when every one of them is bucket-backed
    (summed straight into it), fresh buffers otherwise; returns (buffers, accum)."""
    sinks = [grad_sink(p) for p in params]
    if all(s is not None for s in sinks):
        return sinks, True
    return [torch.empty(sh, dtype=torch.float32, device=dev) for sh in shapes], False


class _ReadoutMLPs(torch.autograd.Function):
    """sum_g mlp_g(feat_g) for the trunk's readouts (readout.py:25-31,42 / 55-62,76, summed in
    model.py:41,50): every readout's Linear+SiLU, Linear+SiLU, Linear(D,1) run as three batched
    launches (blockIdx.y = readout) instead of three per readout, and the sum over readouts is
    fused into the last one; backward likewise (the weight-gradient slab sums deferred)."""

    @staticmethod
    def forward(ctx, G, pool, *args):
        feats, params = args[:G], args[G:]
        W1, B1, W2, B2, W3, B3 = (params[i::6] for i in range(6))
        R, D = feats[0].shape
        ctx.pool = pool
        dev = feats[0].device
        f32 = dict(dtype=torch.float32, device=dev)
        xs = [_f32(f) for f in feats]
        z1 = [torch.empty(R, D, **f32) for _ in range(G)]
        h2 = [torch.empty(R, D, **f32) for _ in range(G)]
        z2 = [torch.empty(R, D, **f32) for _ in range(G)]
        st = stream_ptr()
        ctx.chain = _readout_chain_ok(R, D, G, W1, B1, W2, B2)
        if ctx.chain:  # both hidden layers of every readout: one x2g_chain_fwd_batch launch
            grad = _keeps(ctx)  # inference: no transposed weights, no T-layout inputs
            tf = int(_lib.load().x2g_chain_t_floats(R, D))
            WT = torch.empty(G, 2, D, D, **f32) if grad else None
            in_t = torch.empty(G, 2, tf, **f32) if grad else None

            def wt(g, i):
                return WT[g, i].data_ptr() if grad else None

            stages = [(ChainStage * 2)(ChainStage(_dp(W1[g]), _dp(B1[g]), _dp(z1[g]), None, wt(g, 0), CHAIN_SILU),
                                       ChainStage(_dp(W2[g]), _dp(B2[g]), _dp(z2[g]), _dp(h2[g]), wt(g, 1), CHAIN_SILU))
                      for g in range(G)]
            jobs = (ChainFwdJob * G)(*[ChainFwdJob(_dp(xs[g]), None, ctypes.addressof(stages[g]),
                                                   in_t[g].data_ptr() if grad else None) for g in range(G)])
            call("x2g_chain_fwd_batch", jobs, G, 2, R, D, st)
            heads = (HeadGroup * G)(*[HeadGroup(_dp(h2[g]), _dp(W3[g]), _dp(B3[g]), None, None, None)
                                      for g in range(G)])
            out = _head_fwd(heads, G, R, D, pool, f32, st)
            if grad:
                ctx.save_for_backward(*h2, *z1, *z2, WT, in_t)
            ctx.G, ctx.params = G, params
            return out
        h1 = [torch.empty(R, D, **f32) for _ in range(G)]
        for (src, w, b, y, z) in ((xs, W1, B1, h1, z1), (h1, W2, B2, h2, z2)):
            grp = (DenseFwdGroup * G)(*[DenseFwdGroup(_dp(src[g]), _dp(w[g]), _dp(b[g]), None, _dp(y[g]), _dp(z[g]))
                                        for g in range(G)])
            call("x2g_dense_fwd_batched", grp, G, R, D, D, ACT_SILU, st)
        heads = (HeadGroup * G)(*[HeadGroup(_dp(h2[g]), _dp(W3[g]), _dp(B3[g]), None, None, None) for g in range(G)])
        out = _head_fwd(heads, G, R, D, pool, f32, st)
        ctx.save_for_backward(*xs, *h1, *z1, *h2, *z2)
        ctx.G, ctx.params = G, params
        return out

    @staticmethod
    def backward(ctx, dout):
        G = ctx.G
        saved = ctx.saved_tensors
        if ctx.chain:
            h2, z1, z2 = (saved[i * G:(i + 1) * G] for i in range(3))
            WT, in_t = saved[3 * G], saved[3 * G + 1]
        else:
            xs, h1, z1, h2, z2 = (saved[i * G:(i + 1) * G] for i in range(5))
        W1, B1, W2, B2, W3, B3 = (ctx.params[i::6] for i in range(6))
        R, D = h2[0].shape
        dev = h2[0].device
        f32 = dict(dtype=torch.float32, device=dev)
        lib = _lib.load()
        st = stream_ptr()
        dout = _f32(dout.reshape(-1))
        # head: dh2_g = dout w3_g; dW3_g, db3_g
        dh2 = [torch.empty(R, D, **f32) for _ in range(G)]
        (dw3, db3), acc3 = _wgrad_pairs(W3, B3, dev)
        heads = (HeadGroup * G)(*[HeadGroup(_dp(h2[g]), _dp(W3[g]), None, _dp(dh2[g]), _dp(dw3[g]), _dp(db3[g]))
                                  for g in range(G)])
        ws_bytes = int(lib.x2g_readout_head_bwd_workspace(R, D, G))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        defer = acc3 and _defer() is not None
        hflags = (ACCUM_WGRAD if acc3 else 0) | (DEFER_SLAB_SUM if defer else 0)
        if ctx.pool is not None:  # dout per molecule, broadcast to its rows inside the head kernel
            seg_rowptr, n_seg = ctx.pool
            call("x2g_readout_head_pool_bwd", ptr(dout), ptr(seg_rowptr), n_seg, heads, G, R, D, hflags, ptr(ws),
                 ws_bytes, st)
        else:
            call("x2g_readout_head_bwd", ptr(dout), heads, G, R, D, hflags, ptr(ws), ws_bytes, st)
        if defer:
            splits = int(lib.x2g_readout_head_bwd_splits(R))
            for g in range(G):
                _defer_job(ws, g * splits * (D + 1) * 4, splits, D, 1, dw3[g], db3[g])
        if ctx.chain:  # both hidden layers' data gradients in one launch; dW / db from the T layout
            dfeat = [torch.empty(R, D, **f32) for _ in range(G)]
            dz_t = torch.empty_like(in_t)
            stages = [(ChainBwdStage * 2)(ChainBwdStage(_dp(W1[g]), WT[g, 0].data_ptr(), _dp(z1[g]), None, CHAIN_SILU),
                                          ChainBwdStage(_dp(W2[g]), WT[g, 1].data_ptr(), _dp(z2[g]), None, CHAIN_SILU))
                      for g in range(G)]
            jobs = (ChainBwdJob * G)(*[ChainBwdJob(_dp(dh2[g]), None, ctypes.addressof(stages[g]), _dp(dfeat[g]), None,
                                                   dz_t[g].data_ptr()) for g in range(G)])
            call("x2g_chain_bwd_batch", jobs, G, 2, R, D, st)
            pg = []
            for g in range(G):
                dws, dbs = chain_wgrad(in_t[g], dz_t[g], R, [W1[g], W2[g]], [B1[g], B2[g]])
                pg += [dws[0], dbs[0], dws[1], dbs[1]]
                pg += [None if acc3 else dw3[g].view_as(W3[g]), None if acc3 else db3[g]]
            return (None, None, *dfeat, *pg)
        grads = {}
        # layer 2 then layer 1: dz = dy * SiLU'(z), dx = dz W, dW / db
        dy = dh2
        for (layer, x_in, z, W, B) in ((2, h1, z2, W2, B2), (1, xs, z1, W1, B1)):
            dx = [torch.empty(R, D, **f32) for _ in range(G)]
            (dw, db), acc = _wgrad_pairs(W, B, dev)
            grp = (DenseBwdGroup * G)(*[DenseBwdGroup(_dp(dy[g]), _dp(z[g]), _dp(x_in[g]), _dp(W[g]), _dp(dx[g]), None,
                                                      _dp(dw[g]), _dp(db[g])) for g in range(G)])
            wsz = int(lib.x2g_dense_bwd_workspace(R, D, D))
            ws = torch.empty(max(wsz * G, 1), dtype=torch.uint8, device=dev)
            defer = acc and _defer() is not None
            call("x2g_dense_bwd_batched", grp, G, R, D, D, ACT_SILU, (ACCUM_WGRAD if acc else 0) |
                 (DEFER_SLAB_SUM if defer else 0), ptr(ws), wsz * G, st)
            if defer:
                splits = int(lib.x2g_dense_bwd_splits(R, D, D))
                for g in range(G):
                    _defer_job(ws, g * wsz, splits, D * D, D, dw[g], db[g])
            grads[layer] = (None, None) if acc else (dw, db)
            dy = dx
        dfeat = dy
        pg = []
        for g in range(G):
            for (dw, db) in (grads[1], grads[2]):
                pg += [None if dw is None else dw[g], None if db is None else db[g]]
            pg += [None if acc3 else dw3[g].view_as(W3[g]), None if acc3 else db3[g]]
        return (None, None, *dfeat, *pg)


def _head_fwd(heads, G, R, D, pool, f32, st):
    """sum_g head_g(h_g) -> [R, 1] per row, or [n_seg, 1] summed per segment of rows with the pool
    (x2g_readout_head_pool_fwd: the global add pool fused)."""
    if pool is None:
        out = torch.empty(R, 1, **f32)
        call("x2g_readout_head_fwd", heads, G, R, D, ptr(out), st)
        return out
    seg_rowptr, n_seg = pool
    out = torch.empty(n_seg, 1, **f32)
    call("x2g_readout_head_pool_fwd", heads, G, R, D, ptr(seg_rowptr), n_seg, ptr(out), st)
    return out


# the readouts' two hidden layers as one batched row-chain launch each way (x2g_chain_*_batch) where
# compiled; two batched dense launches each way otherwise
CHAIN_MAX_JOBS = 8  # X2G_CHAIN_MAX_JOBS


class ChainFwdJob(ctypes.Structure):
    """x2g_chain_fwd_job."""
    _fields_ = [("x", ctypes.c_void_p), ("res_ext", ctypes.c_void_p), ("stages", ctypes.c_void_p),
                ("in_t", ctypes.c_void_p)]


class ChainBwdJob(ctypes.Structure):
    """x2g_chain_bwd_job."""
    _fields_ = [("dy", ctypes.c_void_p), ("dy_add", ctypes.c_void_p), ("stages", ctypes.c_void_p),
                ("dx", ctypes.c_void_p), ("d_res_ext", ctypes.c_void_p), ("dz_t", ctypes.c_void_p)]


def _readout_chain_ok(R, D, G, *weights):
    if not _CHAIN or D != 128 or not 1 <= G <= CHAIN_MAX_JOBS or not rows_fit(R, 128):
        return False
    for ws in weights:
        for w in ws:
            if w is not None and (w.dtype != torch.float32 or not w.is_contiguous() or w.data_ptr() % 16):
                return False
    return all(tuple(w.shape) == (128, 128) for ws in (weights[0], weights[2]) for w in ws)


def _wgrad_pairs(Ws, Bs, dev):
    """Weight / bias gradient buffers of a group of layers: the bucket views (accumulate) when all
    are bucket-backed, fresh buffers otherwise."""
    params = list(Ws) + list(Bs)
    bufs, acc = _wgrad_targets(params, [tuple(p.shape) for p in params], dev)
    n = len(Ws)
    return (bufs[:n], bufs[n:]), acc


def readout_mlps_supported(feats, mlps):
    """True when _ReadoutMLPs covers these readouts (same row count and width, the 3-layer
    Linear/SiLU/Linear/SiLU/Linear(D,1) MLP with biases, G <= 8, compiled widths)."""
    from .layers import Linear as _Lin
    G = len(feats)
    if G < 1 or G > 8 or not all(f.is_cuda and f.dim() == 2 and f.shape == feats[0].shape for f in feats):
        return False
    R, D = feats[0].shape
    if D % 4 or D <= 8 or D > 128 or (D // 4) & (D // 4 - 1) or not rows_fit(R, 128):
        return False
    for m in mlps:
        mods = list(m)
        if len(mods) != 5 or not all(isinstance(mods[i], _Lin) for i in (0, 2, 4)):
            return False
        if not all(isinstance(mods[i], torch.nn.SiLU) for i in (1, 3)):
            return False
        if any(mods[i].bias is None for i in (0, 2, 4)):
            return False
        if tuple(mods[0].weight.shape) != (D, D) or tuple(mods[2].weight.shape) != (D, D):
            return False
        if tuple(mods[4].weight.shape) != (1, D):
            return False
    return True


def readout_mlps(feats, mlps, pool=None):
    """sum_g mlp_g(feats[g]) -> [R, 1] (see _ReadoutMLPs); with ``pool = (seg_rowptr int32 [S+1], S)`` the
    rows' sums per segment -> [S, 1] instead (the global add pool after AtomWise, model.py:53, fused into the
    head launch each way)."""
    params = []
    for m in mlps:
        mods = list(m)
        params += [mods[0].weight, mods[0].bias, mods[2].weight, mods[2].bias, mods[4].weight, mods[4].bias]
    if pool is not None:
        pool = (_i32(pool[0]), int(pool[1]))
    return _apply(_ReadoutMLPs, len(feats), pool, *feats, *params)


def keyed_row_sum(src, key, num_keys: int):
    """out[k] = sum of src rows r with key[r] == k (unsorted key): the gradient of table[key]."""
    _need_cuda(src, key)
    src = _f32(src)
    R, D = src.shape
    if num_keys > 16 or D % 4 or D > 256 or (D // 4) & (D // 4 - 1):  # outside the compiled kernel
        onehot = torch.nn.functional.one_hot(key.long(), num_keys).to(torch.float32)
        return linear_wgrad(src, onehot, bias=False)[0].t().contiguous()
    out = torch.empty(num_keys, D, dtype=torch.float32, device=src.device)
    ws_bytes = int(_lib.load().x2g_keyed_row_sum_workspace(R, D, num_keys))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=src.device)
    call("x2g_keyed_row_sum", ptr(src), ptr(_i32(key)), R, D, num_keys, ptr(out), 0, ptr(ws), ws_bytes, stream_ptr())
    return out


# Keyed row sums whose results are only read by the element-table chain's backward (every conv's
# per-destination edge gradient -> its lin_edge table rows): queued here and run as ONE batched
# launch (x2g_keyed_row_sum_batch) when _TableChainFn.backward starts, instead of a partial + a
# slab-sum launch per layer.  The queue belongs to the table chain's forward (one per model call,
# ``table_chain``), not to the module: two models, threads or streams never share it.  False sums
# each immediately.
_DEFER_KEYED = True
KEYED_MAX_JOBS = 8  # X2G_KEYED_MAX_JOBS


def keyed_row_sum_deferred(src, key, num_keys: int, pending: list):
    """keyed_row_sum(src, key, num_keys) into a buffer filled when ``pending`` (the table chain's
    queue) is flushed by flush_keyed(pending)."""
    src = _f32(src)
    R, D = src.shape
    if R == 0 or num_keys > 16 or D % 4 or D > 256 or (D // 4) & (D // 4 - 1):
        return keyed_row_sum(src, key, num_keys)
    out = torch.empty(num_keys, D, dtype=torch.float32, device=src.device)
    pending.append((src, _i32(key), int(num_keys), out))
    return out


def flush_keyed(pending: list):
    """Run every keyed row sum queued on ``pending`` (one partial + one slab-sum launch per group
    of jobs that share keys and shape)."""
    if not pending:
        return
    items = list(pending)
    pending.clear()
    groups = {}
    for src, key, nk, out in items:
        groups.setdefault((key.data_ptr(), tuple(src.shape), nk), []).append((src, key, nk, out))
    lib = _lib.load()
    for (_, (R, D), nk), items in groups.items():
        for j0 in range(0, len(items), KEYED_MAX_JOBS):
            part = items[j0:j0 + KEYED_MAX_JOBS]
            n = len(part)
            srcs = (ctypes.c_void_p * n)(*[it[0].data_ptr() for it in part])
            outs = (ctypes.c_void_p * n)(*[it[3].data_ptr() for it in part])
            wsb = int(lib.x2g_keyed_row_sum_batch_workspace(R, D, nk, n))
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=part[0][0].device)
            call("x2g_keyed_row_sum_batch", srcs, outs, n, ptr(part[0][1]), R, D, nk, 0, ptr(ws), wsb, stream_ptr())


# Inference (grad mode off) with many triplets: S = lin_sbf(sbf) [T, D] is projected and consumed one
# range of destination edges at a time (whole destination segments, at most INFER_TILE triplets),
# so no more than [INFER_TILE, D] of it exists at once.  Sized for 288 GB of HBM: 2^24 triplets are an
# 8.6 GB tile, so config 5 (T = 3.49M, S 1.8 GB per layer) runs whole — one projection and one center
# forward per layer: 8.00 ms per step against 9.11 tiled at 2^19 (seven tiles, 14 launches per layer
# with their ramps and drains; profiles/r5ab_c5_tile.log) and 10.75 at 2^17 (round 4).
INFER_TILE = 1 << 24


def _infer_tiles(lg, tmax):
    """[(e0, e1, t0, t1)] destination-edge ranges of at most ``tmax`` triplets each (a longer
    segment gets a range of its own), cached on the line graph.  With the batch's per-molecule
    counts (``lg.mol_counts``, set by GraphPlan from host metadata) the ranges are whole molecules,
    found without touching the device, so a captured graph can be recorded from a fresh line
    graph; otherwise (the drop-in conv API) from the row pointer, read back once."""
    cache = lg.__dict__.setdefault("_x2g_infer_tiles", {})
    if tmax in cache:
        return cache[tmax]
    counts = getattr(lg, "mol_counts", None)
    ap = None
    if counts is not None:
        ec, tc = counts[0], counts[1]
        ep = np.concatenate([[0], np.cumsum(ec)])
        rp = np.concatenate([[0], np.cumsum(tc)])
        if len(counts) > 2:  # atoms per molecule: each tile's atom range too (center-atom kernels)
            ap = np.concatenate([[0], np.cumsum(counts[2])])
            if ap[-1] != lg.N:
                ap = None
        # the host metadata must describe this line graph, or a tile could split a destination
        # segment or run past E / T: otherwise take the row pointer itself (one read-back)
        if ep[-1] != lg.E or rp[-1] != lg.T or (np.asarray(ec) < 0).any() or (np.asarray(tc) < 0).any():
            counts = None
    if counts is None:
        rp = lg.trip_rowptr.cpu().numpy().astype("int64")
        ep = np.arange(lg.E + 1, dtype=np.int64)
        ap = None
    n = len(rp) - 1
    tiles, i = [], 0
    while i < n:
        j = int(np.searchsorted(rp, rp[i] + tmax, side="right")) - 1  # furthest j with rp[j] - rp[i] <= tmax
        j = min(max(j, i + 1), n)
        if ep[j] > ep[i]:
            atoms = (int(ap[i]), int(ap[j])) if ap is not None else None
            tiles.append((int(ep[i]), int(ep[j]), int(rp[i]), int(rp[j]), atoms))
        i = j
    cache[tmax] = tiles
    return tiles


def _attention_fwd_tiled(q, k, v, skip, edge, sbf, w_sbf, b_sbf, lg, edge_mode, edge_row, heads, channels, tmax,
                         keep_alpha=True):
    q, k, v, skip = _f32(q), _f32(k), _f32(v), _f32(skip)
    sbf, w_sbf, b_sbf = _f32(sbf), _f32(w_sbf), _f32(b_sbf)
    edge = _f32(edge) if edge is not None else None
    E, T, D, H = q.shape[0], lg.T, heads * channels, heads
    f32 = dict(dtype=torch.float32, device=q.device)
    out = torch.empty(E, D, **f32)
    smax, sden = torch.empty(E, H, **f32), torch.empty(E, H, **f32)
    rstats = torch.empty(E, 2, **f32) if _LN_FUSE and D == 128 else None
    tiles = _infer_tiles(lg, tmax)
    materialize_sbf(lg, sbf)
    S = torch.empty(max(t[3] - (t[2] & ~1) for t in tiles), D, **f32)
    st = stream_ptr()
    fb, ib = 4, 4  # bytes per float32 / int32 element
    center, src_row = _center_rows(lg, edge_mode, edge_row, D, channels)
    center = center and all(t[4] is not None for t in tiles)
    alpha = torch.empty(T, H, **f32) if keep_alpha or not center else None  # (the center forward may skip it)
    for e0, e1, t0, t1, atoms in tiles:
        ta = t0 & ~1  # from an even row: the projection's fast path wants 16-byte aligned sbf blocks
        call("x2g_sbf_project", sbf.data_ptr() + ta * sbf.shape[1] * fb, t1 - ta, sbf.shape[1], ptr(w_sbf),
             ptr(b_sbf), D, ptr(S), st)
        if center:  # whole molecules: the tile's atoms own exactly its triplets (S rows t - ta)
            call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(edge), ptr(src_row), edge_mode,
                 ptr(S), ta, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), None, atoms[0], atoms[1] - atoms[0],
                 lg.max_degree, E, T, heads, channels, ptr(out), ptr(alpha), ptr(smax), ptr(sden), ptr(rstats), st)
            continue
        # the kernel reads S at absolute triplet indices t in [t0, t1): hand it the base S - ta rows;
        # everything per destination edge is offset by e0, everything per triplet / per source edge
        # is indexed absolutely
        if edge_mode == EDGE_PER_DST:
            e_edge = ptr(edge) if edge_row is not None else edge.data_ptr() + e0 * D * fb
            e_row = edge_row.data_ptr() + e0 * ib if edge_row is not None else None
        else:
            e_edge, e_row = ptr(edge), None
        call("x2g_sbf_attention_fwd_stats" if rstats is not None else "x2g_sbf_attention_fwd",
             q.data_ptr() + e0 * D * fb, ptr(k), ptr(v), skip.data_ptr() + e0 * D * fb,
             e_edge, e_row, edge_mode, S.data_ptr() - ta * D * fb, None, None, lg.trip_rowptr.data_ptr() + e0 * ib,
             ptr(lg.trip_src), e1 - e0, T, heads, channels, D, out.data_ptr() + e0 * D * fb, ptr(alpha),
             smax.data_ptr() + e0 * H * fb, sden.data_ptr() + e0 * H * fb,
             *((rstats.data_ptr() + e0 * 2 * fb,) if rstats is not None else ()), st)
    return out, alpha, smax, sden, rstats


def sbf_attention(q, k, v, skip, edge, sbf, w_sbf, b_sbf, lg: LineGraph, heads: int, channels: int,
                  edge_mode: int = EDGE_PER_TRIPLET, edge_row=None, return_attention=False):
    """Fused SBFTransformerConv message/softmax/aggregate/skip (see csrc/attention.hip).

    With ``return_attention`` also returns the softmax probabilities [T, heads] (the
    reference's ``return_attention_weights`` alpha)."""
    _need_cuda(q, k, v, skip, sbf)
    if edge is None:
        edge_mode = EDGE_NONE
    if edge_row is not None:
        edge_row = _i32(edge_row)
    sf = (_center_rows(lg, edge_mode, edge_row, heads * channels, channels)[0]
          and _center_sf_ok(lg, _sbf_factors(lg, sbf, edge_mode, heads * channels, edge, edge_row), heads * channels))
    if not torch.is_grad_enabled() and lg.T > INFER_TILE and q.shape[0] > 0 and not sf:  # (sf: no S at all)
        out, alpha, smax, sden, rstats = _attention_fwd_tiled(q, k, v, skip, edge, sbf, w_sbf, b_sbf, lg, edge_mode,
                                                              edge_row, heads, channels, INFER_TILE, return_attention)
    else:
        out, alpha, smax, sden, rstats = _apply(_SBFAttention, q, k, v, skip, edge, sbf, w_sbf, b_sbf, lg, edge_mode,
                                                         edge_row, heads, channels, return_attention)
    if rstats is not None:  # for a graph LayerNorm fused into the consumer (ops.row_chain(ln=...))
        out._x2g_rowstats = rstats
    if not return_attention:
        return out
    dst = lg.trip_dst.long()
    prob = torch.exp(alpha - smax.index_select(0, dst)) / (sden.index_select(0, dst) + 1e-16)
    return out, prob


# ---------------------------------------------------------------------------------- dense layers
ACCUM_WGRAD = 1  # X2G_ACCUM_WGRAD
DEFER_SLAB_SUM = 2  # X2G_DEFER_SLAB_SUM
GATE_DRBF_ACCUM = 4  # X2G_GATE_DRBF_ACCUM


class SlabJob(ctypes.Structure):
    """x2g_slab_job (include/x2g.h)."""
    _fields_ = [("part_w", ctypes.c_void_p), ("part_b", ctypes.c_void_p), ("dw", ctypes.c_void_p),
                ("db", ctypes.c_void_p), ("n_w", ctypes.c_int64), ("n_b", ctypes.c_int32), ("splits", ctypes.c_int32),
                ("ld", ctypes.c_int32), ("cols", ctypes.c_int32)]


class _SlabDeferral:
    """The state of one ``deferred_wgrad()`` context (one backward): the queued slab sums, the
    workspaces they read, the T-layout weight-gradient jobs of the flat launch, and — after the
    context exits — ``flat_launches``: [(rows, cols) per job] of each flat launch it made (bench.py's
    roofline probe replays the largest)."""

    def __init__(self):
        self.jobs = []
        self.keep = []  # workspaces holding the partial slabs until the batched sum is enqueued
        self.tiled = {}  # rows -> [TiledJob]: T-layout weight gradients run as one launch at exit
        self.flat_launches = []


# Open deferrals by HIP stream: autograd runs each backward node on its forward's stream, so a
# backward finds the context its caller opened on that stream, and two models stepping on two
# streams (or threads) never see each other's queue.
_DEFERRALS = {}


def _defer():
    """The deferral open on the current stream, or None."""
    if not _DEFERRALS:
        return None
    return _DEFERRALS.get(torch.cuda.current_stream().cuda_stream)


TILED_MAX_JOBS = 64  # X2G_TILED_MAX_JOBS

# In-step kernel timing for bench.py's roofline line: while a name is a key here, an EAGER (not captured)
# pass appends (start, end) HIP events recorded around that kernel's launch on its stream.  A sleep kernel
# ahead of the start event keeps the device busy while the host enqueues the launch, so the events bracket
# the kernel alone, in the step's own cache state (its operands were just written by the same backward).
KERNEL_TIMERS = {}


@contextlib.contextmanager
def _timed(name):
    evs = KERNEL_TIMERS.get(name)
    if evs is None or torch.cuda.is_current_stream_capturing():
        yield
        return
    st = torch.cuda.current_stream()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # ~0.1 ms of device time ahead of the start event while the host enqueues the launch.  (The eager
    # launch still runs 3-8 % slower than the same launch in graph-replayed steps, box-dependent; a longer
    # sleep or 0.2 ms of matrix work in its place did not change that: DESIGN.md section 5.)
    torch.cuda._sleep(200_000)
    a.record(st)
    yield
    b.record(st)
    evs.append((a, b))


# FLAT_SPLIT > 0: the queued T-layout weight gradients are launched as soon as that many are queued (the
# last layers' group mid-backward, the rest at exit) — the split an exchange overlap needs, so that the
# first group's gradients exist before the backward ends.  0: one flat launch at exit (the default).  A
# constant like the switches above (set explicitly by an A/B script or a test, never from the environment).
FLAT_SPLIT = 0


def _queue_tiled(d, R, jobs, keep):
    """Queue T-layout weight-gradient jobs (x2g_tiled_job, bucket-backed destinations) on deferral
    ``d`` for its flat launch; ``keep``: tensors the jobs point into."""
    d.tiled.setdefault(int(R), []).extend(jobs)
    d.keep.extend(keep)
    if FLAT_SPLIT > 0 and not d.flat_launches and sum(len(j) for j in d.tiled.values()) >= FLAT_SPLIT:
        _flush_tiled(d)


def _flush_tiled(d):
    """Every queued T-layout weight gradient, whatever its row count (the line-node rows of the trunk,
    the atom rows of the readout MLPs), in as few launches as X2G_TILED_MAX_JOBS allows: one at config 2
    (x2g_tiled_wgrad_flat_rows; one launch per row count before).  ``d.flat_launches`` records each
    launch as [(rows, cols) per job]."""
    lib = _lib.load()
    items = [(int(R), j) for R, jobs in d.tiled.items() for j in jobs]
    for j0 in range(0, len(items), TILED_MAX_JOBS):
        part = items[j0:j0 + TILED_MAX_JOBS]
        n = len(part)
        d.flat_launches.append([(R, int(j.cols) if j.ld > 0 else 128) for R, j in part])
        rows = (ctypes.c_int64 * n)(*[R for R, _ in part])
        ws_bytes = int(lib.x2g_tiled_wgrad_flat_rows_workspace(rows, n, 128))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=torch.device("cuda", torch.cuda.current_device()))
        out = (SlabJob * n)()
        jobs = (TiledJob * n)(*[j for _, j in part])
        st = stream_ptr()
        with _timed("tiled_wgrad_flat"):  # (nothing but the launch between the timing events)
            call("x2g_tiled_wgrad_flat_rows", jobs, rows, n, 128, ACCUM_WGRAD | DEFER_SLAB_SUM, out, ptr(ws),
                 ws_bytes, st)
        d.jobs.extend(out)
        d.keep.append(ws)
    d.tiled = {}


@contextlib.contextmanager
def deferred_wgrad():
    """Within this context (on the current stream), weight gradients that go straight into a
    gradient bucket (``grad_sink``) leave their per-workgroup partial slabs in place and the
    T-layout ones are queued; on exit ONE flat weight-gradient launch and ONE x2g_slab_sum_batch
    launch finish every layer's (instead of small launches per layer).  Yields the deferral
    (``flat_launches`` is filled on exit)."""
    key = torch.cuda.current_stream().cuda_stream
    prev = _DEFERRALS.get(key)
    d = _DEFERRALS[key] = _SlabDeferral()
    try:
        yield d
        if d.tiled:
            _flush_tiled(d)
        if d.jobs:
            arr = (SlabJob * len(d.jobs))(*d.jobs)
            call("x2g_slab_sum_batch", ctypes.cast(arr, ctypes.c_void_p), len(d.jobs), 1, stream_ptr())
    finally:
        if prev is None:
            _DEFERRALS.pop(key, None)
        else:
            _DEFERRALS[key] = prev


def _defer_job(ws, offset, splits, n_w, n_b, dw, db, ld=0, cols=0, dw_ptr=None, db_ptr=None, d=None):
    """Queue one slab reduction (x2g_slab_job) on the open deferral; dw_ptr / db_ptr: raw
    destinations (a block of a larger weight) instead of the tensors' own pointers."""
    d = d if d is not None else _defer()
    base = ws.data_ptr() + int(offset)
    has_b = db is not None or db_ptr is not None
    part_b = base + 4 * splits * n_w if has_b else None
    d.jobs.append(SlabJob(base, part_b, dw_ptr if dw_ptr is not None else dw.data_ptr(),
                          (db_ptr if db_ptr is not None else db.data_ptr()) if has_b else None, n_w,
                          n_b if has_b else 0, splits, ld, cols))
    d.keep.append(ws)


_APPLY_GRAD = [True]  # the caller's grad mode at the innermost Function.apply in flight (_apply)


def _apply(fn, *args):
    """``fn.apply(*args)`` with the caller's grad mode recorded for the forward: autograd runs forward() with
    grad mode off and fills ``ctx.needs_input_grad`` from ``requires_grad`` alone, so under ``torch.no_grad()``
    every parameter still "needs" a gradient and a forward that asked only ``needs_input_grad`` kept its
    backward's operands for nothing (config 5's inference wrote ~0.7 GB of logits and P rows and the chains'
    T-layout inputs per layer)."""
    prev = _APPLY_GRAD[0]
    _APPLY_GRAD[0] = torch.is_grad_enabled()
    try:
        return fn.apply(*args)
    finally:
        _APPLY_GRAD[0] = prev


def _keeps(ctx):
    """Whether this forward keeps the operands of a backward: an input needs a gradient AND the caller's
    grad mode was on (see _apply)."""
    return _APPLY_GRAD[0] and any(ctx.needs_input_grad)


def grad_sink(param):
    """The parameter's gradient buffer when the kernels may accumulate into it directly.

    ``dist.GradBucket`` marks its parameters: their ``.grad`` is a view of one flat zeroed buffer,
    so a weight gradient can be summed straight into it by the slab-sum kernel (X2G_ACCUM_WGRAD)
    and the Function returns None for that input — autograd then launches no add kernel for it.
    Unmarked parameters (tests, plain ``loss.backward()``) get their gradient returned as usual."""
    if param is None or not getattr(param, "_x2g_grad_sink", False):
        return None
    g = param.grad
    if g is None or not g.is_contiguous() or g.dtype != torch.float32:
        return None
    return g


class FanIn:
    """In-place gradient fan-in for a tensor every consumer of which is an x2g op that can add its
    share into a buffer (dx_add, X2G_GATE_DRBF_ACCUM, X2G_CHAIN_RES_ACCUM): the first consumer whose
    backward runs writes the buffer and returns it as its gradient, every later one adds into it
    in place and returns None.  Autograd runs the tensor's producer only after ALL consumers, so the
    producer sees the full sum — without the add kernel autograd would launch per extra consumer.

    Attach with ``t._x2g_fanin = FanIn()`` only when every consumer of ``t`` is fan-aware (a plain
    consumer's gradient could be summed with the buffer out of place, and later in-place adds would
    then be lost).  The trunk attaches one per layer input and one to the radial basis."""

    def __init__(self):
        self.buf = None
        self.registered = 0
        self.used = 0

    def register(self):
        self.registered += 1
        return self

    def take(self, shape, device):
        """(buffer, first) for one consumer's backward."""
        first = self.buf is None
        if first:
            self.buf = torch.empty(shape, dtype=torch.float32, device=device)
        buf = self.buf
        self.used += 1
        if self.used >= self.registered:  # the last consumer: the next backward starts afresh
            self.buf, self.used = None, 0
        return buf, first


def _fan_of(t):
    """The FanIn attached to ``t`` (registered as one more consumer), or None."""
    f = getattr(t, "_x2g_fanin", None) if t is not None else None
    return f.register() if f is not None else None


def linear_wgrad(dy, x, bias=True, dw_out=None, db_out=None):
    """(dW [O, I], db [O] or None) with dW = dy^T x, db = column sums of dy, for row-major
    dy [R, O], x [R, I]: row-split MFMA partials + fixed-order slab sum (csrc/linear.hip)."""
    _need_cuda(dy, x)
    dy, x = _f32(dy), _f32(x)
    R, O = dy.shape
    I = x.shape[1]
    accum = dw_out is not None
    if accum and bias and db_out is None:
        raise ValueError("accumulating dW needs the bias-gradient buffer too")
    dw = dw_out if accum else torch.empty(O, I, dtype=torch.float32, device=dy.device)
    db = (db_out if accum else torch.empty(O, dtype=torch.float32, device=dy.device)) if bias else None
    ws_bytes = int(_lib.load().x2g_linear_wgrad_workspace(R, O, I))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dy.device)
    defer = accum and _defer() is not None and R > 0
    flags = (ACCUM_WGRAD if accum else 0) | (DEFER_SLAB_SUM if defer else 0)
    call("x2g_linear_wgrad_ex", ptr(dy), ptr(x), R, O, I, ptr(dw), ptr(db), flags, ptr(ws), ws_bytes, stream_ptr())
    if defer:
        _defer_job(ws, 0, int(_lib.load().x2g_linear_wgrad_splits(R, O, I)), O * I, O, dw, db)
    return (None, None) if accum else (dw, db)


ACT_NONE, ACT_SILU = 0, 1


def _dense_fwd_raw(x2, w, b, act, r2=None, want_z=True):
    """y (and z = pre-activation, when act != none and want_z) for row-major x2 [R, K]."""
    N, K = w.shape
    R = x2.shape[0]
    y = torch.empty(R, N, dtype=torch.float32, device=x2.device)
    z = torch.empty(R, N, dtype=torch.float32, device=x2.device) if (act != ACT_NONE and want_z) else None
    call("x2g_dense_fwd", ptr(x2), ptr(w), ptr(b), R, K, N, act, ptr(r2), ptr(y), ptr(z), stream_ptr())
    return y, z


def _dense_bwd_raw(gy2, z, act, x2, w, w_param, b_param, has_bias, need_dx, dx_add=None, dx_out=None):
    """Fused backward of one dense layer: returns (dx or None, dw or None, db or None).

    dx = dz W (+ dx_add; dx_out may alias dx_add for an in-place accumulation).  Weight grads go
    straight into the flat gradient bucket when the parameters are bucket-backed (grad_sink; then
    (None, None) is returned for them), with their slab sums deferred inside deferred_wgrad()."""
    N, K = w.shape
    R = gy2.shape[0]
    dev = gy2.device
    dx = None
    if need_dx or dx_add is not None:  # (the kernels form dz = dy * act'(z) themselves when dx is not wanted)
        dx = dx_out if dx_out is not None else torch.empty(R, K, dtype=torch.float32, device=dev)
    gw = grad_sink(w_param)
    gb = grad_sink(b_param) if has_bias else None
    accum = gw is not None and (gb is not None or not has_bias)
    if accum:
        dw, db = gw, gb
    else:
        dw = torch.empty(N, K, dtype=torch.float32, device=dev)
        db = torch.empty(N, dtype=torch.float32, device=dev) if has_bias else None
    lib = _lib.load()
    ws_bytes = int(lib.x2g_dense_bwd_workspace(R, K, N))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    defer = accum and _defer() is not None and R > 0
    flags = (ACCUM_WGRAD if accum else 0) | (DEFER_SLAB_SUM if defer else 0)
    call("x2g_dense_bwd_ex", ptr(gy2), ptr(z), act, ptr(x2), ptr(w), R, K, N, ptr(dx), ptr(dx_add), ptr(dw), ptr(db),
         flags, ptr(ws), ws_bytes, stream_ptr())
    if defer:
        _defer_job(ws, lib.x2g_dense_bwd_slab_offset(R, K, N), int(lib.x2g_dense_bwd_splits(R, K, N)), N * K, N, dw,
                   db)
    if accum:
        return dx, None, None
    return dx, dw, db


class _DenseFn(torch.autograd.Function):
    """y = act(x W^T + b) (+ res) in one kernel; backward = one fused kernel (activation
    derivative, data gradient, per-workgroup weight-gradient partials) + a fixed-order slab sum."""

    @staticmethod
    def forward(ctx, x, weight, bias, res, act):
        N, K = weight.shape
        lead = x.shape[:-1]
        x2 = _f32(x.reshape(-1, K))
        w = _f32(weight)
        b = _f32(bias) if bias is not None else None
        r2 = _f32(res.reshape(-1, N)) if res is not None else None
        y, z = _dense_fwd_raw(x2, w, b, act, r2)
        ctx.save_for_backward(x2, w, z)
        ctx.act, ctx.has_bias, ctx.has_res, ctx.lead = act, bias is not None, res is not None, lead
        ctx.w_param, ctx.b_param = weight, bias
        return y.view(*lead, N)

    @staticmethod
    def backward(ctx, gy):
        x2, w, z = ctx.saved_tensors
        N, K = w.shape
        need_x = ctx.needs_input_grad[0]
        dx, dw, db = _dense_bwd_raw(_f32(gy.reshape(-1, N)), z, ctx.act, x2, w, ctx.w_param, ctx.b_param,
                                    ctx.has_bias, need_x)
        dres = gy if ctx.has_res else None
        dx = dx.view(*ctx.lead, K) if need_x else None
        return dx, dw, db, dres, None


class _ResidualFn(torch.autograd.Function):
    """ResidualLayer (residual_layer.py:21-27): y = x + SiLU(W1 SiLU(W0 x + b0) + b1), forward as
    two fused dense kernels; the backward's residual term is folded into the second data
    gradient (dx = dz0 W0 + gy via x2g_dense_bwd_ex's dx_add) instead of an autograd add."""

    @staticmethod
    def forward(ctx, x, w0, b0, w1, b1):
        D = x.shape[-1]
        lead = x.shape[:-1]
        x2 = _f32(x.reshape(-1, D))
        W0, W1 = _f32(w0), _f32(w1)
        B0 = _f32(b0) if b0 is not None else None
        B1 = _f32(b1) if b1 is not None else None
        R = x2.shape[0]
        if W0.shape == (D, D) and W1.shape == (D, D) and D % 4 == 0 and 8 < D <= 128:
            f32 = dict(dtype=torch.float32, device=x2.device)
            h, z0, z1, y = (torch.empty(R, D, **f32) for _ in range(4))
            call("x2g_residual_fwd", ptr(x2), ptr(W0), ptr(B0), ptr(W1), ptr(B1), R, D, ptr(h), ptr(z0), ptr(z1),
                 ptr(y), stream_ptr())
        else:
            h, z0 = _dense_fwd_raw(x2, W0, B0, ACT_SILU)
            y, z1 = _dense_fwd_raw(h, W1, B1, ACT_SILU, r2=x2)
        ctx.save_for_backward(x2, h, z0, z1, W0, W1)
        ctx.params = (w0, b0, w1, b1)
        ctx.lead = lead
        return y.view(*lead, W1.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, h, z0, z1, W0, W1 = ctx.saved_tensors
        w0, b0, w1, b1 = ctx.params
        gy2 = _f32(gy.reshape(-1, W1.shape[0]))
        dh, dw1, db1 = _dense_bwd_raw(gy2, z1, ACT_SILU, h, W1, w1, b1, b1 is not None, True)
        dx, dw0, db0 = _dense_bwd_raw(dh, z0, ACT_SILU, x2, W0, w0, b0, b0 is not None, True, dx_add=gy2)
        return dx.view(*ctx.lead, W0.shape[1]), dw0, db0, dw1, db1


def residual_layer(x, w0, b0, w1, b1):
    if not x.is_cuda:
        raise RuntimeError("x2gnn device ops need GPU tensors (no CPU fallback by design)")
    return _ResidualFn.apply(x, w0, b0, w1, b1)


CHAIN_SILU, CHAIN_HOLD, CHAIN_RES_HELD, CHAIN_RES_EXT = 1, 2, 4, 8  # X2G_CHAIN_* (include/x2g.h)
CHAIN_RES_ACCUM = 16  # backward only
CHAIN_MAX_STAGES = 8


class ChainStage(ctypes.Structure):
    """x2g_chain_stage."""
    _fields_ = [("w", ctypes.c_void_p), ("b", ctypes.c_void_p), ("z", ctypes.c_void_p), ("y", ctypes.c_void_p),
                ("wt", ctypes.c_void_p), ("flags", ctypes.c_int32)]


class ChainBwdStage(ctypes.Structure):
    """x2g_chain_bwd_stage."""
    _fields_ = [("w", ctypes.c_void_p), ("wt", ctypes.c_void_p), ("z", ctypes.c_void_p), ("dz", ctypes.c_void_p),
                ("flags", ctypes.c_int32)]


class WgradJob(ctypes.Structure):
    """x2g_wgrad_job."""
    _fields_ = [("dy", ctypes.c_void_p), ("x", ctypes.c_void_p), ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p)]


def wgrad_batched(dys, xs, weights, biases):
    """Weight / bias gradients of several D x D Linear layers over the same rows in one launch
    (x2g_wgrad_batched): dW_g = dy_g^T x_g, db_g = colsum(dy_g).  Summed straight into the
    gradient bucket when every parameter is bucket-backed (returns Nones for them then), slab sums
    deferred inside ``deferred_wgrad()``; otherwise returns fresh (dW, db) per layer."""
    G = len(dys)
    R, D = dys[0].shape
    dev = dys[0].device
    params = list(weights) + [b for b in biases if b is not None]
    bufs, acc = _wgrad_targets(params, [tuple(p.shape) for p in params], dev)
    dws, rest = bufs[:G], iter(bufs[G:])
    dbs = [next(rest) if b is not None else None for b in biases]
    lib = _lib.load()
    ws_bytes = int(lib.x2g_wgrad_batched_workspace(R, D, G))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    jobs = (WgradJob * G)(*[WgradJob(_dp(dys[g]), _dp(xs[g]), _dp(dws[g]), _dp(dbs[g])) for g in range(G)])
    defer = acc and _defer() is not None
    call("x2g_wgrad_batched", jobs, G, R, D, (ACCUM_WGRAD if acc else 0) | (DEFER_SLAB_SUM if defer else 0), ptr(ws),
         ws_bytes, stream_ptr())
    if defer:
        splits = int(lib.x2g_wgrad_batched_splits(R, D, G))
        per = ws_bytes // G
        for g in range(G):
            _defer_job(ws, g * per, splits, D * D, D, dws[g], dbs[g])
    if acc:
        return [None] * G, [None] * G
    return dws, dbs


def chain_wgrad(in_t, dz_t, R, weights, biases):
    """Weight / bias gradients of every chain stage from the T-layout operands (x2g_chain_wgrad);
    bucket-backed parameters are summed into the bucket (Nones returned for them), slab sums
    deferred inside ``deferred_wgrad()``."""
    n = len(weights)
    D = weights[0].shape[1]
    dev = in_t.device
    params = list(weights) + [b for b in biases if b is not None]
    bufs, acc = _wgrad_targets(params, [tuple(p.shape) for p in params], dev)
    dws, rest = bufs[:n], iter(bufs[n:])
    dbs = [next(rest) if b is not None else None for b in biases]
    d = _defer() if acc else None
    if d is not None:
        tf = in_t.shape[1]
        _queue_tiled(d, R, [TiledJob(dz_t.data_ptr() + 4 * g * tf, in_t.data_ptr() + 4 * g * tf, _dp(dws[g]), _dp(dbs[g]),
                                  0, 0) for g in range(n)], [in_t, dz_t])
        return [None] * n, [None] * n
    lib = _lib.load()
    ws_bytes = int(lib.x2g_chain_wgrad_workspace(R, D, n))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    dw_arr = (ctypes.c_void_p * n)(*[_dp(t) for t in dws])
    db_arr = (ctypes.c_void_p * n)(*[_dp(t) for t in dbs])
    call("x2g_chain_wgrad", ptr(in_t), ptr(dz_t), n, R, D, dw_arr, db_arr, ACCUM_WGRAD if acc else 0, ptr(ws),
         ws_bytes, stream_ptr())
    if acc:
        return [None] * n, [None] * n
    return dws, dbs


class _ChainFn(torch.autograd.Function):
    """A chain of D x D Linear stages on the same rows in ONE kernel (x2g_chain_fwd, csrc/chain.hip):
    stage s computes z_s = in_s W_s^T + b_s, out_s = act(z_s) (+ the held ResidualLayer input or
    the external residual), in_{s+1} = out_s.  Backward: one kernel for every stage's data gradient
    (x2g_chain_bwd, residual gradients folded in registers) + one weight-gradient launch over the
    stage inputs and dz that both kernels leave in the tiled-transposed layout (x2g_chain_wgrad)."""

    @staticmethod
    def forward(ctx, x, res, flags, ln, *params):
        n = len(flags)
        ws, bs = params[0::2], params[1::2]
        x2 = _f32(x)
        R, D = x2.shape
        r2 = _f32(res) if res is not None else None
        f32 = dict(dtype=torch.float32, device=x2.device)
        grad = _keeps(ctx)  # (autograd runs forward() itself with grad mode off: _apply)
        zs = [torch.empty(R, D, **f32) if (flags[i] & CHAIN_SILU) and grad else None for i in range(n)]
        y = torch.empty(R, D, **f32)
        W = [_f32(w) for w in ws]
        B = [_f32(b) if b is not None else None for b in bs]
        tf = int(_lib.load().x2g_chain_t_floats(R, D))
        # for the backward: W^T of every stage, and every stage input in the T layout
        WT = torch.empty(n, D, D, **f32) if grad else None
        in_t = torch.empty(n, tf, **f32) if grad else None
        st = (ChainStage * n)(*[ChainStage(_dp(W[i]), _dp(B[i]), _dp(zs[i]), _dp(y) if i == n - 1 else None,
                                           None if WT is None else WT[i].data_ptr(), flags[i]) for i in range(n)])
        ctx.ln = ln is not None
        if ln is None:
            call("x2g_chain_fwd", ptr(x2), ptr(r2), st, n, R, D, ptr(in_t), stream_ptr())
            ln_saved = ()
        else:  # x is the LayerNorm's input: the chain normalises it while staging
            stats, rowptr, G, eps = ln
            xn = torch.empty(R, D, **f32) if grad else None
            rstd = torch.empty(G, **f32) if grad else None
            call("x2g_chain_fwd_ln", ptr(x2), ptr(stats), ptr(rowptr), G, float(eps), ptr(xn), None, ptr(rstd),
                 ptr(r2), st, n, R, D, ptr(in_t), stream_ptr())
            ln_saved = (xn, rstd, rowptr)
            ctx.ln_segments = G
        if grad:
            ctx.save_for_backward(*W, *[z if z is not None else x2 for z in zs], WT, in_t, *ln_saved)
        ctx.flags, ctx.params, ctx.has_res = tuple(flags), params, res is not None
        ctx.fan_res = _fan_of(res)
        return y

    @staticmethod
    def backward(ctx, gy):
        flags = ctx.flags
        n = len(flags)
        saved = ctx.saved_tensors
        W, zs, WT, in_t = saved[:n], saved[n:2 * n], saved[2 * n], saved[2 * n + 1]
        gy2 = _f32(gy)
        R, D = gy2.shape
        f32 = dict(dtype=torch.float32, device=gy2.device)
        dz_t = torch.empty_like(in_t)
        dx = torch.empty(R, D, **f32)
        dres, first = None, True
        if ctx.has_res and ctx.needs_input_grad[1]:
            if ctx.fan_res is not None:  # add into the layer input's fan-in buffer
                dres, first = ctx.fan_res.take((R, D), gy2.device)
            else:
                dres = torch.empty(R, D, **f32)
        bflags = [f | (CHAIN_RES_ACCUM if (f & CHAIN_RES_EXT) and not first else 0) for f in flags]
        st = (ChainBwdStage * n)(*[ChainBwdStage(_dp(W[i]), WT[i].data_ptr(),
                                                 _dp(zs[i]) if flags[i] & CHAIN_SILU else None, None, bflags[i])
                                   for i in range(n)])
        if not ctx.ln:
            call("x2g_chain_bwd", ptr(gy2), None, st, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), stream_ptr())
        elif _LN_BWD_ROWS:  # dx is the LayerNorm output's gradient: through its backward to the chain's input,
            # the per-row sums it needs left by the chain's last store
            xn, rstd, rowptr = saved[2 * n + 2:2 * n + 5]
            gst = torch.empty(R, 2, **f32)
            call("x2g_chain_bwd_ln", ptr(gy2), None, st, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), ptr(xn), ptr(gst),
                 stream_ptr())
            dxp = torch.empty(R, D, **f32)
            call("x2g_graph_layernorm_bwd_rows", ptr(xn), ptr(dx), ptr(rstd), ptr(rowptr), ctx.ln_segments, D, ptr(gst),
                 ptr(dxp), stream_ptr())
            dx = dxp
        else:
            call("x2g_chain_bwd", ptr(gy2), None, st, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), stream_ptr())
            xn, rstd, rowptr = saved[2 * n + 2:2 * n + 5]
            G = ctx.ln_segments
            dxp = torch.empty(R, D, **f32)
            wsb = int(_lib.load().x2g_graph_layernorm_bwd_workspace(G))
            lws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=gy2.device)
            call("x2g_graph_layernorm_bwd_ex", ptr(xn), ptr(dx), ptr(rstd), ptr(rowptr), G, D, ptr(dxp), ptr(lws), wsb,
                 stream_ptr())
            dx = dxp
        ws, bs = ctx.params[0::2], ctx.params[1::2]
        dws, dbs = chain_wgrad(in_t, dz_t, R, ws, bs)
        grads = []
        for i in range(n):
            grads += [dws[i], dbs[i]]
        return (dx, dres if first else None, None, None, *grads)


def chain_supported(x, linears):
    """True when _ChainFn's kernels cover these layers (D = 128 rows of 16-byte aligned fp32)."""
    if not x.is_cuda or x.dim() != 2 or x.shape[1] != 128 or not rows_fit(x.shape[0], 128):
        return False
    if len(linears) < 1 or len(linears) > CHAIN_MAX_STAGES:
        return False
    for m in linears:
        if tuple(m.weight.shape) != (128, 128) or m.weight.dtype != torch.float32 or m.weight.data_ptr() % 16:
            return False
        if m.bias is not None and m.bias.data_ptr() % 16:
            return False
    return True


_CHAIN = True  # False: layer-by-layer dense kernels (tests/test_gpu_kernels.py flips it)


def row_chain(x, res, linears, flags, ln=None):
    """Apply the chain of ``linears`` (nn.Linear modules, D x D) with per-stage X2G_CHAIN_* flags.

    ``ln`` = (row_stats [R, 2], segment rowptr [G + 1] int32, G, eps): the chain's input is the
    graph LayerNorm of x (model.py:46), computed while staging from the per-row (mean, M2) the
    attention forward left (``x._x2g_rowstats``); the backward runs the LayerNorm's too."""
    params = []
    for m in linears:
        params += [m.weight, m.bias]
    if ln is not None:
        stats, rowptr, G, eps = ln
        ln = (_f32(stats), _i32(rowptr), int(G), float(eps))
    return _apply(_ChainFn, x, res, tuple(flags), ln, *params)


# ------------------------------------------------------------------------------ small-table chains
TABLE_MAX_STAGES = 8  # X2G_TABLE_MAX_STAGES
_FAN_IN = True  # False: autograd's own fan-in adds (test_fan_in_gradients_match_autograd_adds)


class TableStage(ctypes.Structure):
    """x2g_table_stage."""
    _fields_ = [("w", ctypes.c_void_p), ("b", ctypes.c_void_p), ("parent", ctypes.c_int32), ("act", ctypes.c_int32),
                ("z", ctypes.c_void_p), ("y", ctypes.c_void_p)]


class TableBwdStage(ctypes.Structure):
    """x2g_table_bwd_stage."""
    _fields_ = [("w", ctypes.c_void_p), ("in_", ctypes.c_void_p), ("z", ctypes.c_void_p), ("dy", ctypes.c_void_p),
                ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p), ("parent", ctypes.c_int32), ("act", ctypes.c_int32),
                ("accum", ctypes.c_int32)]


def table_chain_supported(x, linears):
    """True when x2g_table_chain_* cover these layers: D = 128, <= 16 rows, aligned fp32 weights."""
    if not x.is_cuda or x.dim() != 2 or x.shape[1] != 128 or x.shape[0] > 16:
        return False
    if not 1 <= len(linears) <= TABLE_MAX_STAGES:
        return False
    for m in linears:
        if tuple(m.weight.shape) != (128, 128) or m.weight.dtype != torch.float32 or m.weight.data_ptr() % 16:
            return False
        if m.bias is not None and (m.bias.dtype != torch.float32 or m.bias.data_ptr() % 16):
            return False
    return True


class _TableChainFn(torch.autograd.Function):
    """A tree of D x D Linear stages on a <= 16-row table (x2g_table_chain_fwd/bwd): stage s reads
    x (parent -1) or an earlier stage's output; one launch per direction for the whole tree."""

    @staticmethod
    def forward(ctx, x, spec, pending, *params):
        n = len(spec)
        x2 = _f32(x).contiguous()
        R, D = x2.shape
        dev = x2.device
        ws = [_f32(p).contiguous() for p in params[0::2]]
        bs = [_f32(p).contiguous() if p is not None else None for p in params[1::2]]
        f32 = dict(dtype=torch.float32, device=dev)
        ys = [torch.empty(R, D, **f32) for _ in range(n)]
        zs = [torch.empty(R, D, **f32) if spec[s][1] == ACT_SILU else None for s in range(n)]
        st = (TableStage * n)(*[TableStage(_dp(ws[s]), _dp(bs[s]), spec[s][0], spec[s][1], _dp(zs[s]), _dp(ys[s]))
                                for s in range(n)])
        call("x2g_table_chain_fwd", ptr(x2), R, D, st, n, stream_ptr())
        ctx.save_for_backward(x2, *ws, *ys, *zs)
        ctx.spec, ctx.params, ctx.pending = spec, params, pending
        ctx.set_materialize_grads(False)
        return tuple(ys)

    @staticmethod
    def backward(ctx, *gys):
        flush_keyed(ctx.pending)  # the conv layers' deferred edge-table gradients (keyed_row_sum_deferred)
        spec, n = ctx.spec, len(ctx.spec)
        saved = ctx.saved_tensors
        x2, ws, ys, zs = saved[0], saved[1:1 + n], saved[1 + n:1 + 2 * n], saved[1 + 2 * n:1 + 3 * n]
        R, D = x2.shape
        dev = x2.device
        dys = [_f32(g).contiguous() if g is not None else None for g in gys]
        grads, stages = [], []
        for s in range(n):
            wp, bp = ctx.params[2 * s], ctx.params[2 * s + 1]
            gw = grad_sink(wp)
            gb = grad_sink(bp) if bp is not None else None
            accum = gw is not None and (bp is None or gb is not None)
            if accum:
                dw, db = gw, gb
                grads += [None, None]
            else:
                dw = torch.empty(D, D, dtype=torch.float32, device=dev)
                db = torch.empty(D, dtype=torch.float32, device=dev) if bp is not None else None
                grads += [dw, db]
            par, act = spec[s]
            src = x2 if par < 0 else ys[par]
            stages.append(TableBwdStage(_dp(ws[s]), _dp(src), _dp(zs[s]), _dp(dys[s]), _dp(dw), _dp(db), par, act,
                                        1 if accum else 0))
        dx = torch.empty(R, D, dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        # several leaves (the four lin_edge): leaf stages side by side, then the inner ones
        wsb = int(_lib.load().x2g_table_chain_bwd_workspace(n))
        ws = torch.empty(max(wsb, 16), dtype=torch.uint8, device=dev)
        call("x2g_table_chain_bwd_ex", (TableBwdStage * n)(*stages), n, R, D, ptr(dx), ptr(ws), wsb, stream_ptr())
        return (dx, None, None, *grads)


def table_chain(x, stages):
    """Outputs of every stage of ``stages`` = [(Linear, act, parent), ...] applied to the table x."""
    params, spec = [], []
    for m, act, parent in stages:
        params += [m.weight, m.bias]
        spec.append((int(parent), int(act)))
    pending = []  # keyed row sums consumers queue for this chain's backward (keyed_row_sum_deferred)
    outs = _TableChainFn.apply(x, tuple(spec), pending, *params)
    for o in outs:
        o._x2g_keyed_pending = pending
    return outs


# --------------------------------------------------------------------------- line-node featurisation
def featurize_supported(x, env, lin1, lin2):
    """True when x2g_feat_fwd/bwd cover SiLU(lin2(SiLU(lin1(x * env)))): x [R, K] fp32 with
    256 < K <= 384 even and no gradient wanted for x / env, lin1 K -> 256, lin2 256 -> 128."""
    if not x.is_cuda or x.dim() != 2 or x.dtype != torch.float32 or x.requires_grad:
        return False
    R, K = x.shape
    if not (256 < K <= 384 and K % 2 == 0) or not rows_fit(R, 384):
        return False
    if env is not None and (env.numel() != R or env.requires_grad):
        return False
    if tuple(lin1.weight.shape) != (256, K) or tuple(lin2.weight.shape) != (128, 256):
        return False
    for p in (lin1.weight, lin1.bias, lin2.weight, lin2.bias):
        if p is not None and (p.dtype != torch.float32 or p.data_ptr() % 16):
            return False
    return True


class _FeaturizeFn(torch.autograd.Function):
    """neo_x = SiLU(W2 SiLU(W1 (x * env) + b1) + b2) (xgnn.py:64-67): one forward kernel, one
    backward data kernel and one 8-job T-layout weight-gradient launch (csrc/feature.hip)."""

    @staticmethod
    def forward(ctx, x, env, w1, b1, w2, b2):
        x2 = _f32(x)
        R, K = x2.shape
        dev = x2.device
        tf = int(_lib.load().x2g_chain_t_floats(R, 128))
        f32 = dict(dtype=torch.float32, device=dev)
        y = torch.empty(R, 128, **f32)
        # the backward's T-layout operands (8 planes, ~4 KB per row) only when a gradient is wanted
        grad = _keeps(ctx)
        xs_t, z1_t, y1_t, z2_t = ((torch.empty(max(n * tf, 1), **f32) for n in (3, 2, 2, 1)) if grad
                                  else (None, None, None, None))
        e = _f32(env.reshape(-1)) if env is not None else None
        W1, W2 = _f32(w1), _f32(w2)
        B1 = _f32(b1) if b1 is not None else None
        B2 = _f32(b2) if b2 is not None else None
        call("x2g_feat_fwd", ptr(x2), ptr(e), R, K, ptr(W1), ptr(B1), ptr(W2), ptr(B2), ptr(y), ptr(xs_t), ptr(z1_t),
             ptr(y1_t), ptr(z2_t), stream_ptr())
        if grad:
            ctx.save_for_backward(xs_t, z1_t, y1_t, z2_t, W2)
        ctx.R, ctx.K, ctx.tf = R, K, tf
        ctx.params = (w1, b1, w2, b2)
        return y

    @staticmethod
    def backward(ctx, gy):
        xs_t, z1_t, y1_t, z2_t, W2 = ctx.saved_tensors
        R, K, tf = ctx.R, ctx.K, ctx.tf
        dev = gy.device
        f32 = dict(dtype=torch.float32, device=dev)
        dz2_t, dz1_t = torch.empty(max(tf, 1), **f32), torch.empty(max(2 * tf, 1), **f32)
        call("x2g_feat_bwd", ptr(_f32(gy)), ptr(z2_t), ptr(z1_t), ptr(W2), R, ptr(dz2_t), ptr(dz1_t), stream_ptr())
        w1, b1, w2, b2 = ctx.params
        params = [p for p in (w1, b1, w2, b2) if p is not None]
        bufs, acc = _wgrad_targets(params, [tuple(p.shape) for p in params], dev)
        it = iter(bufs)
        dw1 = next(it)
        db1 = next(it) if b1 is not None else None
        dw2 = next(it)
        db2 = next(it) if b2 is not None else None
        fb = 4  # bytes per float
        specs = []  # (dy_t, x_t, dw pointer, db pointer, ld, cols)
        for o in range(2):
            for i in range(3):
                specs.append((dz1_t.data_ptr() + fb * o * tf, xs_t.data_ptr() + fb * i * tf,
                              dw1.data_ptr() + fb * (o * 128 * K + i * 128),
                              db1.data_ptr() + fb * o * 128 if (db1 is not None and i == 0) else None, K,
                              min(128, K - 128 * i)))
        for i in range(2):
            specs.append((dz2_t.data_ptr(), y1_t.data_ptr() + fb * i * tf, dw2.data_ptr() + fb * i * 128,
                          db2.data_ptr() if (db2 is not None and i == 0) else None, 256, 128))
        n = len(specs)
        d = _defer() if acc else None
        if d is not None:
            _queue_tiled(d, R, [TiledJob(*sp) for sp in specs], [dz1_t, dz2_t, xs_t, y1_t])
            return None, None, None, None, None, None
        lib = _lib.load()
        ws_bytes = int(lib.x2g_tiled_wgrad_workspace(R, 128, n))
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        jobs = (TiledJob * n)(*[TiledJob(*sp) for sp in specs])
        call("x2g_tiled_wgrad", jobs, n, R, 128, ACCUM_WGRAD if acc else 0, ptr(ws), ws_bytes, stream_ptr())
        if acc:
            return None, None, None, None, None, None
        return None, None, dw1, db1, dw2, db2


def featurize(x, env, lin1, lin2):
    """SiLU(lin2(SiLU(lin1(x * env[:, None])))) through the fused featurisation kernels."""
    return _apply(_FeaturizeFn, x, env, lin1.weight, lin1.bias, lin2.weight, lin2.bias)


class TiledJob(ctypes.Structure):
    """x2g_tiled_job."""
    _fields_ = [("dy_t", ctypes.c_void_p), ("x_t", ctypes.c_void_p), ("dw", ctypes.c_void_p), ("db", ctypes.c_void_p),
                ("ld", ctypes.c_int32), ("cols", ctypes.c_int32)]


class Proj(ctypes.Structure):
    """x2g_proj."""
    _fields_ = [("w", ctypes.c_void_p), ("b", ctypes.c_void_p), ("out", ctypes.c_void_p), ("wt", ctypes.c_void_p)]


class ProjGrad(ctypes.Structure):
    """x2g_proj_grad."""
    _fields_ = [("g", ctypes.c_void_p), ("w", ctypes.c_void_p), ("wt", ctypes.c_void_p), ("g_t", ctypes.c_void_p)]


def tiled_wgrad(dy_ts, x_ts, R, weights, biases):
    """Weight / bias gradients of D x D Linear layers from T-layout operands (x2g_tiled_wgrad), one
    job per layer; bucket-backed parameters are summed into the bucket (Nones returned), slab sums
    deferred inside ``deferred_wgrad()``."""
    n = len(weights)
    D = weights[0].shape[1]
    dev = dy_ts[0].device
    params = list(weights) + [b for b in biases if b is not None]
    bufs, acc = _wgrad_targets(params, [tuple(p.shape) for p in params], dev)
    dws, rest = bufs[:n], iter(bufs[n:])
    dbs = [next(rest) if b is not None else None for b in biases]
    d = _defer() if acc else None
    if d is not None:
        _queue_tiled(d, R, [TiledJob(_dp(dy_ts[g]), _dp(x_ts[g]), _dp(dws[g]), _dp(dbs[g]), 0, 0) for g in range(n)],
                     list(dy_ts) + list(x_ts))
        return [None] * n, [None] * n
    lib = _lib.load()
    ws_bytes = int(lib.x2g_tiled_wgrad_workspace(R, D, n))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    jobs = (TiledJob * n)(*[TiledJob(_dp(dy_ts[g]), _dp(x_ts[g]), _dp(dws[g]), _dp(dbs[g])) for g in range(n)])
    call("x2g_tiled_wgrad", jobs, n, R, D, ACCUM_WGRAD if acc else 0, ptr(ws), ws_bytes, stream_ptr())
    if acc:
        return [None] * n, [None] * n
    return dws, dbs


def conv_proj_fused_supported(x, rbf, weights, biases):
    """True when the row-chain style projection kernels (x2g_conv_proj_fwd / _bwd) cover the layer."""
    if not _CHAIN or not x.is_cuda or x.dim() != 2 or x.shape[1] != 128 or not rows_fit(x.shape[0], 128):
        return False
    if rbf.dim() != 2 or not 1 <= rbf.shape[1] <= 8 or rbf.shape[0] != x.shape[0]:
        return False
    for w in weights:
        if tuple(w.shape) != (128, 128) or w.dtype != torch.float32 or w.data_ptr() % 16:
            return False
    return all(b is None or b.data_ptr() % 16 == 0 for b in biases)


def _conv_proj_bwd_gate(grads, x2, rbf2, Wr, wr, dx, first_x, need_rbf, drbf_out, first_r):
    """x2g_conv_proj_bwd_gate: dx (in place, += when not first_x), drbf, dW_rbf of the projections'
    backward in one launch; returns (dx, drbf, dW_rbf) with None where the gradient went into a
    caller's buffer (fan-in, gradient bucket)."""
    E, D = x2.shape
    RR = rbf2.shape[1]
    dev = x2.device
    drbf = drbf_out if drbf_out is not None else (
        torch.empty(E, RR, dtype=torch.float32, device=dev) if need_rbf else None)
    gw = grad_sink(wr)
    accum = gw is not None
    dw = gw if accum else torch.empty(D, RR, dtype=torch.float32, device=dev)
    lib = _lib.load()
    ws_bytes = int(lib.x2g_conv_proj_bwd_gate_workspace(E, RR))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    defer = accum and _defer() is not None and E > 0
    flags = ((ACCUM_WGRAD if accum else 0) | (DEFER_SLAB_SUM if defer else 0)
             | (GATE_DRBF_ACCUM if (need_rbf and not first_r) else 0))
    call("x2g_conv_proj_bwd_gate", grads, E, D, ptr(x2), ptr(rbf2), RR, ptr(Wr), ptr(dx),
         None if first_x else ptr(dx), ptr(drbf), ptr(dw), flags, ptr(ws), ws_bytes, stream_ptr())
    if defer:
        _defer_job(ws, 0, int(lib.x2g_conv_proj_bwd_gate_splits(E)), D * RR, 0, dw, None)
    return dx, drbf, (None if accum else dw)


class _ConvProjFusedFn(torch.autograd.Function):
    """SBFTransformerConv's projections (sbftransformer_conv.py:99-107,127) in one kernel each way:
    x2g_conv_proj_fwd (x and x_src = x * lin_rbf(rbf) in LDS, q/k/v/skip per wave slice) and
    x2g_conv_proj_bwd (dx = dq Wq + dskip Ws, dx_src = dk Wk + dv Wv) + the gate backward
    (x2g_rbf_gate_bwd: dx += dx_src * f, drbf, dW_rbf) + one T-layout weight-gradient launch."""

    @staticmethod
    def forward(ctx, x, rbf, wr, wq, bq, wk, bk, wv, bv, ws, bs):
        E, D = x.shape
        x2, rbf2, Wr = _f32(x), _f32(rbf), _f32(wr)
        W = [_f32(t) for t in (wq, wk, wv, ws)]
        B = [_f32(t) if t is not None else None for t in (bq, bk, bv, bs)]
        f32 = dict(dtype=torch.float32, device=x2.device)
        outs = [torch.empty(E, D, **f32) for _ in range(4)]
        grad = _keeps(ctx)
        lib = _lib.load()
        tf = int(lib.x2g_chain_t_floats(E, D))
        WT = torch.empty(4, D, D, **f32) if grad else None
        x_t = torch.empty(tf, **f32) if grad else None
        xs_t = torch.empty(tf, **f32) if grad else None
        proj = (Proj * 4)(*[Proj(_dp(W[i]), _dp(B[i]), _dp(outs[i]), None if WT is None else WT[i].data_ptr())
                            for i in range(4)])
        call("x2g_conv_proj_fwd", ptr(x2), ptr(rbf2), rbf2.shape[1], ptr(Wr), proj, E, D, ptr(x_t), ptr(xs_t),
             stream_ptr())
        if grad:
            ctx.save_for_backward(x2, rbf2, Wr, *W, WT, x_t, xs_t)
        ctx.params = (wr, wq, bq, wk, bk, wv, bv, ws, bs)
        ctx.fan_x, ctx.fan_r = _fan_of(x), _fan_of(rbf)
        return tuple(outs)

    @staticmethod
    def backward(ctx, gq, gk, gv, gskip):
        x2, rbf2, Wr, Wq, Wk, Wv, Ws, WT, x_t, xs_t = ctx.saved_tensors
        wr, wq, bq, wk, bk, wv, bv, ws, bs = ctx.params
        E, D = x2.shape
        f32 = dict(dtype=torch.float32, device=x2.device)
        g = [_f32(t) if t is not None else torch.zeros(E, D, **f32) for t in (gq, gk, gv, gskip)]
        tf = x_t.shape[0]
        g_t = torch.empty(4, tf, **f32)
        W = (Wq, Wk, Wv, Ws)
        grads = (ProjGrad * 4)(*[ProjGrad(_dp(g[i]), _dp(W[i]), WT[i].data_ptr(), g_t[i].data_ptr())
                                 for i in range(4)])
        first_x = first_r = True
        if ctx.fan_x is not None:  # dx goes into (or adds onto) the layer input's fan-in buffer
            dx, first_x = ctx.fan_x.take((E, D), x2.device)
        else:
            dx = torch.empty(E, D, **f32)
        need_rbf = ctx.needs_input_grad[1]
        drbf_out = None
        if need_rbf and ctx.fan_r is not None:
            drbf_out, first_r = ctx.fan_r.take(rbf2.shape, x2.device)
        # the gate's backward inside the projection kernel: dxs stays in registers
        gx, grbf, dwr = _conv_proj_bwd_gate(grads, x2, rbf2, Wr, wr, dx, first_x, need_rbf, drbf_out, first_r)
        gx = gx if first_x else None
        grbf = grbf if first_r else None
        dws, dbs = tiled_wgrad([g_t[0], g_t[1], g_t[2], g_t[3]], [x_t, xs_t, xs_t, x_t], E, [wq, wk, wv, ws],
                               [bq, bk, bv, bs])
        return (gx, (grbf if need_rbf else None), dwr, dws[0], dbs[0], dws[1], dbs[1], dws[2], dbs[2], dws[3],
                dbs[3])


class _ConvProjFn(torch.autograd.Function):
    """The dense projections of SBFTransformerConv.forward (sbftransformer_conv.py:99-107,127):
    rf = lin_rbf(rbf), x_src = x * rf, q = lin_query(x), k = lin_key(x_src), v = lin_value(x_src),
    skip = lin_skip(x).  The backward chains the four data gradients into one buffer per input
    (x2g_dense_bwd_ex dx_add, in place) instead of summing them with autograd adds."""

    @staticmethod
    def forward(ctx, x, rbf, wr, wq, bq, wk, bk, wv, bv, ws, bs):
        E, D = x.shape
        x2, rbf2 = _f32(x), _f32(rbf)
        Wr, Wq, Wk, Wv, Ws = (_f32(t) for t in (wr, wq, wk, wv, ws))
        Bq, Bk, Bv, Bs = (_f32(t) if t is not None else None for t in (bq, bk, bv, bs))
        if gate_supported(D, rbf2.shape[1]):  # x_src = x * lin_rbf(rbf), filter not materialised
            rf = None
            xs = torch.empty_like(x2)
            call("x2g_rbf_gate_fwd", ptr(x2), ptr(rbf2), ptr(Wr), None, E, D, rbf2.shape[1], ptr(xs), stream_ptr())
        else:
            rf, _ = _dense_fwd_raw(rbf2, Wr, None, ACT_NONE)
            xs = x2 * rf
        q, k, v, skip = _projections4(x2, xs, (Wq, Bq), (Wk, Bk), (Wv, Bv), (Ws, Bs))
        ctx.save_for_backward(x2, rbf2, rf, xs, Wr, Wq, Wk, Wv, Ws)  # rf None on the gate path
        ctx.params = (wr, wq, bq, wk, bk, wv, bv, ws, bs)
        return q, k, v, skip

    @staticmethod
    def backward(ctx, gq, gk, gv, gskip):
        x2, rbf2, rf, xs, Wr, Wq, Wk, Wv, Ws = ctx.saved_tensors
        wr, wq, bq, wk, bk, wv, bv, ws, bs = ctx.params
        g = [_f32(t) if t is not None else torch.zeros_like(x2) for t in (gq, gk, gv, gskip)]
        gxs, dwk, dbk = _dense_bwd_raw(g[1], None, ACT_NONE, xs, Wk, wk, bk, bk is not None, True)
        gxs, dwv, dbv = _dense_bwd_raw(g[2], None, ACT_NONE, xs, Wv, wv, bv, bv is not None, True, dx_add=gxs,
                                       dx_out=gxs)
        need_rbf = ctx.needs_input_grad[1]
        if rf is None:  # one pass: gx = gxs * f, grbf, dWr
            gx, grbf, dwr, _ = _gate_bwd(gxs, None, x2, rbf2, Wr, None, wr, None, True, need_rbf)
        else:
            grf = gxs * x2  # d rf
            gx = gxs * rf   # x_src = x * rf
        gx, dwq, dbq = _dense_bwd_raw(g[0], None, ACT_NONE, x2, Wq, wq, bq, bq is not None, True, dx_add=gx,
                                      dx_out=gx)
        gx, dws, dbs = _dense_bwd_raw(g[3], None, ACT_NONE, x2, Ws, ws, bs, bs is not None, True, dx_add=gx,
                                      dx_out=gx)
        if rf is not None:
            grbf, dwr, _ = _dense_bwd_raw(grf, None, ACT_NONE, rbf2, Wr, wr, None, False, need_rbf)
        return gx, (grbf if need_rbf else None), dwr, dwq, dbq, dwk, dbk, dwv, dbv, dws, dbs


def _projections4(x2, xs, pq, pk, pv, ps):
    """q = lin_query(x), k = lin_key(x_src), v = lin_value(x_src), skip = lin_skip(x) as ONE
    batched launch (x2g_dense_fwd_batched, 4 groups) when the shapes allow, else four."""
    R, K = x2.shape
    N = pq[0].shape[0]
    outs = [torch.empty(R, N, dtype=torch.float32, device=x2.device) for _ in range(4)]
    ok = (K % 4 == 0 and N % 4 == 0 and 8 < K <= 128 and N <= 128 and rows_fit(R, 128)
          and all(p[0].shape == pq[0].shape for p in (pk, pv, ps)))
    if ok and R > 0:
        srcs = (x2, xs, xs, x2)
        grp = (DenseFwdGroup * 4)(*[DenseFwdGroup(_dp(srcs[g]), _dp(p[0]), _dp(p[1]), None, _dp(outs[g]), None)
                                    for g, p in enumerate((pq, pk, pv, ps))])
        call("x2g_dense_fwd_batched", grp, 4, R, K, N, ACT_NONE, stream_ptr())
        return outs
    return [_dense_fwd_raw(src, p[0], p[1], ACT_NONE)[0] for src, p in zip((x2, xs, xs, x2), (pq, pk, pv, ps))]


def gate_supported(D, R):
    """Shapes the rbf-gate kernels are compiled for (csrc/rbf_gate.hip)."""
    return D in (64, 128, 256) and 1 <= R <= 8


def _gate_bwd(g, owner, x, rbf, w, b, w_param, b_param, need_dx, need_rbf, dx_add=None, dx_out=None, drbf_out=None,
              drbf_acc=False):
    """x2g_rbf_gate_bwd: (dx, drbf, dw, db); dw / db are None when summed into the gradient bucket.
    dx_out / drbf_out: caller buffers (dx_out may alias dx_add); drbf_acc: drbf_out += the gradient."""
    rows, D = x.shape
    R = rbf.shape[1]
    dev = x.device
    dx = dx_out if dx_out is not None else (torch.empty(rows, D, dtype=torch.float32, device=dev) if need_dx else None)
    drbf = drbf_out if drbf_out is not None else (
        torch.empty(rows, R, dtype=torch.float32, device=dev) if need_rbf else None)
    has_bias = b is not None
    gw, gb = grad_sink(w_param), (grad_sink(b_param) if has_bias else None)
    accum = gw is not None and (gb is not None or not has_bias)
    if accum:
        dw, db = gw, gb
    else:
        dw = torch.empty(D, R, dtype=torch.float32, device=dev)
        db = torch.empty(D, dtype=torch.float32, device=dev) if has_bias else None
    lib = _lib.load()
    ws_bytes = int(lib.x2g_rbf_gate_bwd_workspace(rows, D, R))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    defer = accum and _defer() is not None and rows > 0
    flags = (ACCUM_WGRAD if accum else 0) | (DEFER_SLAB_SUM if defer else 0) | (GATE_DRBF_ACCUM if drbf_acc else 0)
    call("x2g_rbf_gate_bwd", ptr(g), ptr(owner), ptr(x), ptr(rbf), ptr(w), ptr(b), rows, D, R, ptr(dx), ptr(dx_add),
         ptr(drbf), ptr(dw), ptr(db), flags, ptr(ws), ws_bytes, stream_ptr())
    if defer:
        _defer_job(ws, 0, int(lib.x2g_rbf_gate_bwd_splits(rows)), D * R, D, dw, db)
    return dx, drbf, (None if accum else dw), (None if accum else db)


class _RbfPoolFn(torch.autograd.Function):
    """out[n] = sum over rows e of segment n of x[e] * (W rbf[e] + b) (readout.py:39-41,66-67:
    lin_rbf(rbf) * x pooled edges -> atoms) without the [E, D] filter tensor."""

    @staticmethod
    def forward(ctx, x, rbf, w, b, owner, rowptr, n_seg):
        x2, rbf2, W = _f32(x), _f32(rbf), _f32(w)
        B = _f32(b) if b is not None else None
        D, R = x2.shape[1], rbf2.shape[1]
        out = torch.empty(n_seg, D, dtype=torch.float32, device=x2.device)
        call("x2g_rbf_pool_fwd", ptr(x2), ptr(rbf2), ptr(W), ptr(B), ptr(rowptr), n_seg, D, R, ptr(out), stream_ptr())
        ctx.save_for_backward(x2, rbf2, W, B)
        ctx.owner, ctx.params = owner, (w, b)
        ctx.fan_x, ctx.fan_r = _fan_of(x), _fan_of(rbf)
        return out

    @staticmethod
    def backward(ctx, gp):
        x2, rbf2, W, B = ctx.saved_tensors
        w, b = ctx.params
        need_x, need_r = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dev = x2.device
        dx_out = drbf_out = None
        first_x = first_r = True
        if need_x and ctx.fan_x is not None:
            dx_out, first_x = ctx.fan_x.take(x2.shape, dev)
        if need_r and ctx.fan_r is not None:
            drbf_out, first_r = ctx.fan_r.take(rbf2.shape, dev)
        dx, drbf, dw, db = _gate_bwd(_f32(gp), ctx.owner, x2, rbf2, W, B, w, b, need_x, need_r,
                                     dx_add=None if first_x else dx_out, dx_out=dx_out, drbf_out=drbf_out,
                                     drbf_acc=not first_r)
        return (dx if first_x else None), (drbf if first_r else None), dw, db, None, None, None


def _addr(t):
    """Raw device address of a tensor for a ctypes struct field (None -> NULL)."""
    return None if t is None else t.data_ptr()


class GateJob(ctypes.Structure):
    """x2g_gate_job."""
    _fields_ = [("x", ctypes.c_void_p), ("w", ctypes.c_void_p), ("b", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("g", ctypes.c_void_p), ("dx", ctypes.c_void_p), ("dx_add", ctypes.c_void_p), ("dw", ctypes.c_void_p),
                ("db", ctypes.c_void_p)]


GATE_MAX_JOBS = 8  # X2G_GATE_MAX_JOBS
# the readouts' edge -> atom pools as one launch each way (x2g_rbf_pool_fwd_batch / _gate_bwd_batch)
_POOL_BATCH = True


class _RbfPoolBatchFn(torch.autograd.Function):
    """Several rbf pools over the same rows / atoms / basis (_RbfPoolFn's math per job), one launch
    each way; the basis gradient is the jobs' sum (one fan-in consumer for the whole batch)."""

    @staticmethod
    def forward(ctx, n, rbf, owner, rowptr, n_seg, *tensors):
        xs, ws, bs = tensors[:n], tensors[n:2 * n], tensors[2 * n:]
        rbf2 = _f32(rbf)
        x2 = [_f32(x) for x in xs]
        W = [_f32(w) for w in ws]
        B = [_f32(b) if b is not None else None for b in bs]
        D, R = x2[0].shape[1], rbf2.shape[1]
        outs = [torch.empty(n_seg, D, dtype=torch.float32, device=rbf2.device) for _ in range(n)]
        jobs = (GateJob * n)(*[GateJob(x2[j].data_ptr(), W[j].data_ptr(), _addr(B[j]), outs[j].data_ptr(), None, None,
                                       None, None, None) for j in range(n)])
        call("x2g_rbf_pool_fwd_batch", jobs, n, ptr(rbf2), ptr(rowptr), n_seg, D, R, stream_ptr())
        ctx.save_for_backward(rbf2, *x2, *W)
        ctx.n, ctx.n_seg, ctx.B, ctx.owner, ctx.params = n, n_seg, B, owner, (ws, bs)
        ctx.fan_x = [_fan_of(x) for x in xs]
        ctx.fan_r = _fan_of(rbf)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gps):
        n = ctx.n
        saved = ctx.saved_tensors
        rbf2, x2, W = saved[0], saved[1:1 + n], saved[1 + n:1 + 2 * n]
        ws, bs = ctx.params
        rows, D = x2[0].shape
        R = rbf2.shape[1]
        dev = rbf2.device
        need_r = ctx.needs_input_grad[1]
        drbf, first_r = None, True
        if need_r:
            if ctx.fan_r is not None:
                drbf, first_r = ctx.fan_r.take(rbf2.shape, dev)
            else:
                drbf = torch.empty(rows, R, dtype=torch.float32, device=dev)
        dx_ret, jobs, keep, sinks = [], [], [], []
        for j in range(n):
            need_x = ctx.needs_input_grad[5 + j]
            dx, first = None, True
            if need_x:
                if ctx.fan_x[j] is not None:
                    dx, first = ctx.fan_x[j].take(x2[j].shape, dev)
                else:
                    dx = torch.empty(rows, D, dtype=torch.float32, device=dev)
            dx_ret.append(dx if (need_x and first) else None)
            has_b = ctx.B[j] is not None
            gw, gb = grad_sink(ws[j]), (grad_sink(bs[j]) if has_b else None)
            accum = gw is not None and (gb is not None or not has_b)
            if not accum:
                gw = torch.empty(D, R, dtype=torch.float32, device=dev)
                gb = torch.empty(D, dtype=torch.float32, device=dev) if has_b else None
            sinks.append((accum, gw, gb))
            g = _f32(gps[j]) if gps[j] is not None else torch.zeros(ctx.n_seg, D, dtype=torch.float32, device=dev)
            keep.append(g)
            jobs.append(GateJob(x2[j].data_ptr(), W[j].data_ptr(), _addr(ctx.B[j]), None, g.data_ptr(), _addr(dx),
                                None if first else _addr(dx), gw.data_ptr(), _addr(gb)))
        accums = {a for a, _, _ in sinks}
        if len(accums) != 1:
            raise RuntimeError("rbf_pool_batch: mixed bucket / plain weight gradients in one batch")
        accum = accums.pop()
        lib = _lib.load()
        ws_bytes = int(lib.x2g_rbf_gate_bwd_batch_workspace(rows, D, R, n))
        wsb = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        d = _defer() if accum else None
        defer = d is not None
        flags = (ACCUM_WGRAD if accum else 0) | (DEFER_SLAB_SUM if defer else 0) | (0 if first_r else GATE_DRBF_ACCUM)
        out = (SlabJob * n)()
        call("x2g_rbf_gate_bwd_batch", (GateJob * n)(*jobs), n, ptr(ctx.owner), ptr(rbf2), rows, D, R, ptr(drbf), flags,
             out, ptr(wsb), ws_bytes, stream_ptr())
        if defer:
            d.jobs.extend(out)
            d.keep.append(wsb)
        dws = [None if accum else gw for _, gw, _ in sinks]
        dbs = [None if accum else gb for _, _, gb in sinks]
        return (None, drbf if (need_r and first_r) else None, None, None, None, *dx_ret, *dws, *dbs)


def rbf_pool_batch(xs, rbf, weights, biases, owner, rowptr, n_seg: int):
    """[rbf_pool(x_j, rbf, W_j, b_j, owner, rowptr, n_seg) for j] in one launch each way."""
    _need_cuda(rbf, *xs)
    n = len(xs)
    return list(_RbfPoolBatchFn.apply(n, rbf, _i32(owner), _i32(rowptr), int(n_seg), *xs, *weights, *biases))


def rbf_pool_batch_supported(xs, rbf, weights):
    return (_POOL_BATCH and 1 < len(xs) <= GATE_MAX_JOBS and all(x.is_cuda and x.dim() == 2 for x in xs)
            and len({tuple(x.shape) for x in xs}) == 1 and gate_supported(xs[0].shape[1], rbf.shape[1])
            and all(tuple(w.shape) == (xs[0].shape[1], rbf.shape[1]) for w in weights))


def rbf_pool(x, rbf, weight, bias, owner, rowptr, n_seg: int):
    """Segment sums of x * lin_rbf(rbf) over rows sorted by ``owner`` (CSR ``rowptr``)."""
    _need_cuda(x, rbf)
    return _RbfPoolFn.apply(x, rbf, weight, bias, _i32(owner), _i32(rowptr), int(n_seg))


def conv_projections(x, rbf, wr, wq, bq, wk, bk, wv, bv, ws, bs):
    if not x.is_cuda:
        raise RuntimeError("x2gnn device ops need GPU tensors (no CPU fallback by design)")
    if conv_proj_fused_supported(x, rbf, (wq, wk, wv, ws), (bq, bk, bv, bs)):
        return _apply(_ConvProjFusedFn, x, rbf, wr, wq, bq, wk, bk, wv, bv, ws, bs)
    return _apply(_ConvProjFn, x, rbf, wr, wq, bq, wk, bk, wv, bv, ws, bs)


def dense(x, weight, bias=None, act=ACT_NONE, res=None):
    """Fused row-wise Linear (+ SiLU) (+ residual) on the GPU (csrc/dense.hip)."""
    if not x.is_cuda:
        raise RuntimeError("x2gnn device ops need GPU tensors (no CPU fallback by design)")
    return _DenseFn.apply(x, weight, bias, res, act)


def linear(x, weight, bias=None):
    return dense(x, weight, bias)


# ---------------------------------------------------------------------------------- segments
def _seg_sum_raw(x, mul, rowptr, n_seg):
    D = x.shape[1]
    out = torch.empty(n_seg, D, dtype=torch.float32, device=x.device)
    call("x2g_segment_sum", ptr(x), ptr(mul), ptr(rowptr), n_seg, D, ptr(out), stream_ptr())
    return out


def _seg_bcast_raw(g, mul, rowptr, n_rows):
    D = g.shape[1]
    out = torch.empty(n_rows, D, dtype=torch.float32, device=g.device)
    call("x2g_segment_broadcast", ptr(g), ptr(mul), ptr(rowptr), g.shape[0], D, ptr(out), stream_ptr())
    return out


class _SegmentSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mul, rowptr, n_seg):
        x = _f32(x)
        mul = _f32(mul) if mul is not None else None
        ctx.save_for_backward(x, mul, rowptr)
        return _seg_sum_raw(x, mul, rowptr, n_seg)

    @staticmethod
    def backward(ctx, g):
        x, mul, rowptr = ctx.saved_tensors
        g = _f32(g)
        dx = _seg_bcast_raw(g, mul, rowptr, x.shape[0]) if ctx.needs_input_grad[0] else None
        dmul = None
        if mul is not None and ctx.needs_input_grad[1]:
            dmul = _seg_bcast_raw(g, x, rowptr, x.shape[0])
        return dx, dmul, None, None


def segment_sum(x, rowptr, num_segments: int, mul=None):
    """out[g] = sum_{r in segment g} x[r] (* mul[r]); rows of a segment are contiguous."""
    _need_cuda(x, rowptr)
    squeeze = x.dim() == 1
    if squeeze:
        x = x.unsqueeze(1)
        mul = mul.unsqueeze(1) if mul is not None else None
    out = _SegmentSum.apply(x, mul, _i32(rowptr), int(num_segments))
    return out.squeeze(1) if squeeze else out


class IndexPlan:
    """A scatter index in any order, prepared on the device without a host read: ``perm`` is the
    stable sort of the keys (sorted position -> source row; equal keys keep the caller's order) and
    ``rowptr`` the CSR row pointer of the sorted keys.  Rows whose key lies outside [0, dim_size)
    belong to no segment (torch_scatter raises for them).  Build once, reuse for every operator
    over the same index (as MessagePassing reuses edge_index[1])."""

    def __init__(self, index, dim_size: int):
        _need_cuda(index)
        idx = _i32(index.reshape(-1))
        self.n, self.dim_size = int(idx.numel()), int(dim_size)
        keys, perm = torch.sort(idx, stable=True)
        self.perm = _i32(perm)
        self.rowptr, _ = csr_rowptr_checked(keys, self.dim_size)


REDUCE_SUM, REDUCE_MEAN = 0, 1  # X2G_REDUCE_*


class _ScatterReduce(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, plan, mode):
        x = _f32(src)
        out = torch.empty(plan.dim_size, x.shape[1], dtype=torch.float32, device=x.device)
        call("x2g_segment_reduce_perm", ptr(x), ptr(plan.perm), ptr(plan.rowptr), plan.dim_size, x.shape[1], mode,
             ptr(out), stream_ptr())
        ctx.plan, ctx.mode, ctx.rows = plan, mode, x.shape[0]
        return out

    @staticmethod
    def backward(ctx, g):
        g = _f32(g)
        plan = ctx.plan
        dx = torch.zeros(ctx.rows, g.shape[1], dtype=torch.float32, device=g.device)
        call("x2g_segment_reduce_perm_bwd", ptr(g), ptr(plan.perm), ptr(plan.rowptr), plan.dim_size, g.shape[1],
             ctx.mode, ptr(dx), stream_ptr())
        return dx, None, None


def _plan_rows(src, plan):
    """A prebuilt IndexPlan's row count must be src's: its permutation addresses src's rows."""
    _need_cuda(src)
    if src.shape[0] != plan.n:
        raise ValueError(f"IndexPlan was built for {plan.n} rows, src has {src.shape[0]}")


def _scatter(src, index, dim_size, mode):
    if isinstance(index, IndexPlan):
        _plan_rows(src, index)
        if dim_size is not None and int(dim_size) != index.dim_size:
            raise ValueError(f"dim_size {dim_size} differs from the IndexPlan's {index.dim_size}")
        plan = index
    else:
        _need_cuda(src, index)
        if src.shape[0] != index.numel():
            raise ValueError("scatter: index must hold one key per row of src (dim=0)")
        if dim_size is None:  # torch_scatter's default: index.max() + 1 (a host read)
            dim_size = int(index.max()) + 1 if index.numel() else 0
        plan = IndexPlan(index, int(dim_size))
    squeeze = src.dim() == 1
    x = src.unsqueeze(1) if squeeze else src.reshape(src.shape[0], -1)
    out = _ScatterReduce.apply(x, plan, mode)
    return out.squeeze(1) if squeeze else out.view(plan.dim_size, *src.shape[1:])


def scatter_add(src, index, dim_size: int = None):
    """torch_scatter.scatter_add(src, index, dim=0, dim_size=dim_size) (readout.py:37, model.py:53)
    for ANY index order (or a prebuilt ``IndexPlan``), with no host read (HIP-graph capturable):
    the keys are stably sorted on the device and the segment sum reads src's rows through the
    permutation (x2g_segment_reduce_perm), so each segment is summed in the caller's row order —
    deterministic, no float atomics."""
    return _scatter(src, index, dim_size, REDUCE_SUM)


def scatter_mean(src, index, dim_size: int = None):
    """torch_scatter.scatter_mean(src, index, dim=0, dim_size=dim_size) (readout.py:69, MolWise's
    pool_option='mean'): the segment sum divided by max(count, 1), empty segments 0; any index order,
    no host read."""
    return _scatter(src, index, dim_size, REDUCE_MEAN)


class _SegmentSoftmax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, rowptr, n_seg):
        src = _f32(src)
        out = torch.empty_like(src)
        call("x2g_segment_softmax_fwd", ptr(src), ptr(rowptr), n_seg, src.shape[1], ptr(out), stream_ptr())
        ctx.save_for_backward(out, rowptr)
        ctx.n_seg = n_seg
        return out

    @staticmethod
    def backward(ctx, g):
        out, rowptr = ctx.saved_tensors
        g = _f32(g)
        ds = torch.empty_like(out)
        call("x2g_segment_softmax_bwd", ptr(out), ptr(g), ptr(rowptr), ctx.n_seg, out.shape[1], ptr(ds), stream_ptr())
        return ds, None, None


def segment_softmax(src, rowptr, num_segments: int):
    """PyG utils.softmax for a sorted index, [R] or [R, H]."""
    _need_cuda(src, rowptr)
    squeeze = src.dim() == 1
    s = src.unsqueeze(1) if squeeze else src
    out = _SegmentSoftmax.apply(s, _i32(rowptr), int(num_segments))
    return out.squeeze(1) if squeeze else out


class _SoftmaxPerm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, src, plan):
        x = _f32(src)
        out = torch.empty_like(x)
        call("x2g_segment_softmax_perm_fwd", ptr(x), ptr(plan.perm), ptr(plan.rowptr), plan.dim_size, x.shape[1],
             ptr(out), stream_ptr())
        ctx.save_for_backward(out)
        ctx.plan = plan
        return out

    @staticmethod
    def backward(ctx, g):
        (out,) = ctx.saved_tensors
        plan = ctx.plan
        ds = torch.zeros_like(out)
        call("x2g_segment_softmax_perm_bwd", ptr(out), ptr(_f32(g)), ptr(plan.perm), ptr(plan.rowptr), plan.dim_size,
             out.shape[1], ptr(ds), stream_ptr())
        return ds, None


def softmax(src, index=None, ptr=None, num_nodes=None):
    """torch_geometric.utils.softmax(src, index, ptr, num_nodes) along dim 0
    (sbftransformer_conv.py:151): exp(src - max) / (sum + 1e-16) per group of rows sharing a key.
    ``index`` in any order (or an ``IndexPlan``), or a CSR ``ptr`` of contiguous groups.  With
    neither ``num_nodes`` nor an IndexPlan the group count is ``int(index.max()) + 1`` (a host read,
    as PyG's maybe_num_nodes makes); otherwise nothing is read back."""
    if ptr is not None:
        return segment_softmax(src, ptr, int(ptr.numel()) - 1)
    if index is None:
        raise ValueError("softmax needs index or ptr")
    if isinstance(index, IndexPlan):
        _plan_rows(src, index)
    else:
        _need_cuda(src, index)
        if src.shape[0] != index.numel():
            raise ValueError("softmax: index must hold one key per row of src (dim=0)")
        n = int(num_nodes) if num_nodes is not None else (int(index.max()) + 1 if index.numel() else 0)
        index = IndexPlan(index, n)
    squeeze = src.dim() == 1
    s = src.unsqueeze(1) if squeeze else src
    out = _SoftmaxPerm.apply(s, index)
    return out.squeeze(1) if squeeze else out


class _GraphLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, rowptr, n_seg, eps):
        x = _f32(x)
        D = x.shape[1]
        out = torch.empty_like(x)
        mean = torch.empty(n_seg, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        call("x2g_graph_layernorm_fwd", ptr(x), ptr(rowptr), n_seg, D, float(eps), ptr(out), ptr(mean), ptr(rstd),
             stream_ptr())
        ctx.save_for_backward(out, rstd, rowptr)
        ctx.n_seg = n_seg
        return out

    @staticmethod
    def backward(ctx, g):
        out, rstd, rowptr = ctx.saved_tensors
        g = _f32(g)
        dx = torch.empty_like(out)
        wsb = int(_lib.load().x2g_graph_layernorm_bwd_workspace(ctx.n_seg))
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=out.device)
        call("x2g_graph_layernorm_bwd_ex", ptr(out), ptr(g), ptr(rstd), ptr(rowptr), ctx.n_seg, out.shape[1], ptr(dx),
             ptr(ws), wsb, stream_ptr())
        return dx, None, None, None


def graph_layer_norm(x, rowptr, num_segments: int, eps: float = 1e-5):
    """PyG LayerNorm(mode='graph', affine=False) over contiguous row segments."""
    _need_cuda(x, rowptr)
    return _GraphLayerNorm.apply(x, _i32(rowptr), int(num_segments), float(eps))


# ------------------------------------------------------------------------------ loss
class _SmoothL1MeanFn(torch.autograd.Function):
    """F.smooth_l1_loss(pred, target) with reduction='mean' (trainer.py:41) as one launch each way
    (x2g_smooth_l1_mean_fwd / _bwd) instead of torch's elementwise + mean and fill + fill +
    elementwise; the target takes no gradient (the reference's labels)."""

    @staticmethod
    def forward(ctx, pred, target, beta, unit_seed):
        p, t = _f32(pred).reshape(-1), _f32(target).reshape(-1)
        out = torch.empty((), dtype=torch.float32, device=p.device)
        ctx.unit_seed, ctx.dp_unit = unit_seed, None
        if unit_seed is not None:  # the gradient for a backward seeded with `unit_seed` (== 1) in the same pass
            ctx.dp_unit = torch.empty_like(p)
            call("x2g_smooth_l1_mean_fwd_grad", ptr(p), ptr(t), p.numel(), float(beta), ptr(out), ptr(ctx.dp_unit),
                 stream_ptr())
        else:
            call("x2g_smooth_l1_mean_fwd", ptr(p), ptr(t), p.numel(), float(beta), ptr(out), stream_ptr())
        ctx.save_for_backward(p, t)
        ctx.beta, ctx.shape = float(beta), pred.shape
        return out

    @staticmethod
    def backward(ctx, g):
        if ctx.dp_unit is not None and g is ctx.unit_seed:  # autograd hands the caller's seed object through
            return ctx.dp_unit.view(ctx.shape), None, None, None
        p, t = ctx.saved_tensors
        dp = torch.empty_like(p)
        call("x2g_smooth_l1_mean_bwd", ptr(p), ptr(t), p.numel(), ctx.beta, ptr(_f32(g).reshape(1)), ptr(dp),
             stream_ptr())
        return dp.view(ctx.shape), None, None, None


def smooth_l1_loss(pred, target, beta: float = 1.0, unit_seed=None):
    """torch.nn.functional.smooth_l1_loss(pred, target, beta=beta) (mean) on the device path.

    ``unit_seed``: a persistent ones scalar the caller will pass to ``torch.autograd.backward(loss,
    unit_seed)`` (x2gnn.train.Trainer's ``seed``): the forward launch then also writes the gradient for
    that seed, and the backward, handed that very object, returns it without a launch (any other
    gradient takes the backward kernel, so the result is the same either way, bit for bit)."""
    if (not pred.is_cuda or pred.shape != target.shape or pred.numel() == 0 or target.requires_grad
            or beta <= 0):  # beta <= 0 is torch's L1 branch, not compiled
        return torch.nn.functional.smooth_l1_loss(pred, target, beta=beta)
    return _SmoothL1MeanFn.apply(pred, target, beta, unit_seed)
