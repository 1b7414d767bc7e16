"""SBFTransformerConv on the line graph, backed by the fused gfx950 attention kernels.

Same constructor and ``forward(sbf, rbf, x, edge_index, edge_attr)`` contract as the
reference (sbftransformer_conv.py:16-166, a PyG ``MessagePassing`` with aggr='add'):

    x_src = x * lin_rbf(rbf);  q = lin_query(x);  k, v = lin_key(x_src), lin_value(x_src)
    per triplet t = (src -> dst):  e_t = lin_edge(edge_attr_t)
        alpha_t = softmax_dst( <q[dst], k[src] + e_t> / sqrt(C) )          (per head)
        m_t     = (v[src] + e_t) * lin_sbf(sbf_t) * alpha_t
    out[dst] = sum_t m_t  (+ lin_skip(x) with root_weight)

The five projections (lin_rbf gate, q/k/v/skip) run as one fused f32-MFMA kernel each way
(``ops.conv_projections``; the generic dense kernels for widths outside the compiled set).
``lin_sbf(sbf)`` is materialised once per layer as S [T, H*C] (``x2g_sbf_project``), and
everything else per triplet (gathers, logits, softmax, the weighted sum, the skip add) runs in
one destination-major kernel (``ops.sbf_attention``); the backward folds lin_sbf's gradient per
source line node instead of writing a [T, H*C] gradient (csrc/attention_fold.inc).

Triplets may come in any order (PyG's ``propagate`` accepts any).  By default the destinations
are stably sorted on the device and the per-triplet inputs permuted alike — no host read, so the
call is HIP-graph capturable; the attention weights, when requested, come back in the caller's
order.  ``assume_sorted=True`` (the order vertex_to_edge_2 emits, edge_graph.py:12-30) skips the
sort and its gathers; the order is then checked on the device and a violation is flagged on the
line graph (``LineGraph.order_violated()``), never an out-of-range access.

Extra keyword-only arguments for the in-framework fast path:
``line_graph`` (a prebuilt ``ops.LineGraph``), ``edge_row`` (when ``edge_attr`` is a small
table and triplets into line node e use row ``edge_row[e]``: X2-GNN's edge attribute is the
embedding of the middle atom, identical for all triplets into e, xgnn.py:57-58) and
``edge_proj`` (``lin_edge(edge_attr)`` already computed, e.g. by the trunk's table chain).
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch
import torch.nn as nn

from . import ops
from .layers import Linear


class SBFTransformerConv(nn.Module):
    def __init__(self, in_channels: Union[int, Tuple[int, int]], out_channels: int, heads: int = 1,
                 sbf_dim: int = 16, rbf_dim: int = 16, concat: bool = True, beta: bool = False,
                 dropout: float = 0.0, edge_dim: Optional[int] = None, bias: bool = True,
                 root_weight: bool = True, **kwargs):
        super().__init__()
        if not concat or (beta and root_weight):
            raise NotImplementedError("compiled configuration: concat=True, beta=False (X2-GNN's)")
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.sbf_dim, self.rbf_dim = sbf_dim, rbf_dim
        self.beta, self.root_weight, self.concat = False, root_weight, concat
        self.dropout, self.edge_dim = dropout, edge_dim
        cin = (in_channels, in_channels) if isinstance(in_channels, int) else tuple(in_channels)
        hc = heads * out_channels
        self.lin_key = Linear(cin[0], hc)
        self.lin_query = Linear(cin[1], hc)
        self.lin_value = Linear(cin[0], hc)
        self.lin_edge = Linear(edge_dim, hc, bias=False) if edge_dim is not None else None
        self.lin_skip = Linear(cin[1], hc, bias=bias)
        self.lin_beta = None
        self.lin_sbf = Linear(sbf_dim, hc, bias=True)
        self.lin_rbf = Linear(rbf_dim, cin[0], bias=False)
        self._alpha = None

    def forward(self, sbf, rbf, x, edge_index, edge_attr=None, return_attention_weights=None, *,
                line_graph: Optional[ops.LineGraph] = None, edge_row=None, edge_proj=None,
                assume_sorted: bool = False):
        H, C = self.heads, self.out_channels
        if self.training and self.dropout > 0:
            raise NotImplementedError("attention dropout is not compiled (X2-GNN uses dropout=0)")
        if x.is_cuda and self.root_weight and x.dim() == 2:
            # one autograd node for the five projections: the backward chains the data
            # gradients into one buffer per input instead of autograd adds
            q, k, v, skip = ops.conv_projections(
                x, rbf, self.lin_rbf.weight, self.lin_query.weight, self.lin_query.bias, self.lin_key.weight,
                self.lin_key.bias, self.lin_value.weight, self.lin_value.bias, self.lin_skip.weight, self.lin_skip.bias)
        else:
            x_src = x * self.lin_rbf(rbf)
            q = self.lin_query(x)
            k = self.lin_key(x_src)
            v = self.lin_value(x_src)
            skip = self.lin_skip(x) if self.root_weight else torch.zeros_like(q)
        perm = None
        if line_graph is None:
            dst = edge_index[1]
            if not assume_sorted and dst.numel() > 1:
                # CSR by destination needs dst-sorted triplets: stable device sort, the per-triplet
                # inputs follow (identity for an already sorted index; no host read either way)
                perm = torch.argsort(dst, stable=True)
                edge_index = edge_index.index_select(1, perm)
                sbf = sbf.index_select(0, perm)
                if edge_attr is not None and edge_row is None and edge_proj is None:
                    edge_attr = edge_attr.index_select(0, perm)
                if edge_proj is not None and edge_row is None:
                    edge_proj = edge_proj.index_select(0, perm)
            line_graph = ops.LineGraph.from_triplets(edge_index, x.shape[0])
        if edge_proj is not None:  # lin_edge(edge_attr) computed by the caller (the trunk's table chain)
            e = edge_proj
            mode = ops.EDGE_PER_DST if edge_row is not None else ops.EDGE_PER_TRIPLET
        elif edge_attr is not None and self.lin_edge is not None:
            e = self.lin_edge(edge_attr)
            mode = ops.EDGE_PER_DST if edge_row is not None else ops.EDGE_PER_TRIPLET
        else:
            e, mode = None, ops.EDGE_NONE
        want = isinstance(return_attention_weights, bool)
        res = ops.sbf_attention(q, k, v, skip, e, sbf, self.lin_sbf.weight, self.lin_sbf.bias, line_graph, H, C,
                                edge_mode=mode, edge_row=edge_row, return_attention=want)
        if want:
            out, alpha = res
            if perm is not None:  # back to the caller's triplet order
                alpha = torch.empty_like(alpha).index_copy_(0, perm, alpha)
                edge_index = torch.empty_like(edge_index).index_copy_(1, perm, edge_index)
            return out, (edge_index, alpha)
        return res

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels}, heads={self.heads})"

