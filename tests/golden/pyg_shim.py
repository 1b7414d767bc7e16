"""Test infrastructure: restated PyG 2.1.0 / torch_scatter 2.1.0 semantics for importing the
reference in THIS container only (they are not installed).

Only the entry points X2-GNN reaches are restated:

* ``torch_scatter.scatter_add / scatter_mean / scatter`` — sum into ``dim_size`` rows, empty
  segments 0; mean divides by the count clamped to >= 1; ``reduce='max'`` fills empty rows with 0.
* ``torch_geometric.utils.softmax(src, index, ptr=None, num_nodes=None)`` — segment max shift,
  ``exp``, divide by (segment sum + 1e-16).
* ``torch_geometric.nn.LayerNorm(in_channels, eps, affine, mode='graph')`` — per-graph mean /
  variance over all (rows x channels) of the graph, ``x / sqrt(var + eps)``.
* ``torch_geometric.nn.conv.MessagePassing`` — ``propagate`` lifts ``*_i`` by
  ``edge_index[1]`` and ``*_j`` by ``edge_index[0]`` (``index_select``), passes ``index``
  (= edge_index[1]), ``ptr=None``, ``size_i``, then sum-aggregates by ``index``.
* ``torch_geometric.nn.dense.linear.Linear`` — ``F.linear`` with ``weight[out,in]``/``bias``.
* ``torch_geometric.data.Data`` — attribute bag with ``_store``.
"""
from __future__ import annotations

import inspect
import math
import sys
import types

import torch
import torch.nn.functional as F


def scatter_add(src, index, dim=-1, out=None, dim_size=None):
    dim = dim % src.dim()
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() else 0
    shape = list(src.shape)
    shape[dim] = dim_size
    res = torch.zeros(shape, dtype=src.dtype, device=src.device)
    return res.index_add(dim, index.long(), src)


def scatter_mean(src, index, dim=-1, out=None, dim_size=None):
    dim = dim % src.dim()
    s = scatter_add(src, index, dim, dim_size=dim_size)
    cnt = scatter_add(torch.ones(src.shape[dim], dtype=src.dtype), index, 0, dim_size=s.shape[dim])
    cnt = cnt.clamp(min=1)
    view = [1] * s.dim()
    view[dim] = -1
    return s / cnt.view(view)


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    dim = dim % src.dim()
    if reduce in ("sum", "add"):
        return scatter_add(src, index, dim, dim_size=dim_size)
    if reduce == "mean":
        return scatter_mean(src, index, dim, dim_size=dim_size)
    if reduce == "max":
        assert dim == 0
        if dim_size is None:
            dim_size = int(index.max()) + 1
        idx = index.long().view(-1, *([1] * (src.dim() - 1))).expand_as(src)
        res = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype)
        return res.scatter_reduce(0, idx, src, reduce="amax", include_self=False)
    raise ValueError(reduce)


def softmax(src, index=None, ptr=None, num_nodes=None, dim=0):
    assert ptr is None and index is not None and dim == 0
    n = int(index.max()) + 1 if num_nodes is None else num_nodes
    src_max = scatter(src, index, 0, dim_size=n, reduce="max").index_select(0, index)
    out = (src - src_max).exp()
    out_sum = scatter(out, index, 0, dim_size=n, reduce="sum").index_select(0, index)
    return out / (out_sum + 1e-16)


def degree(index, num_nodes=None, dtype=None):
    n = int(index.max()) + 1 if num_nodes is None else num_nodes
    out = torch.zeros(n, dtype=dtype or torch.long)
    return out.index_add(0, index, torch.ones(index.numel(), dtype=out.dtype))


def remove_self_loops(edge_index, edge_attr=None):
    mask = edge_index[0] != edge_index[1]
    return edge_index[:, mask], (None if edge_attr is None else edge_attr[mask])


class Data:
    def __init__(self, **kwargs):
        object.__setattr__(self, "_store", {})
        for k, v in kwargs.items():
            if v is not None:
                self._store[k] = v

    def __getattr__(self, key):
        st = object.__getattribute__(self, "_store")
        if key in st:
            return st[key]
        raise AttributeError(key)

    def __setattr__(self, key, value):
        self._store[key] = value


class Linear(torch.nn.Module):
    def __init__(self, in_channels, out_channels, bias=True, weight_initializer=None,
                 bias_initializer=None):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = torch.nn.Parameter(torch.empty(out_channels, in_channels))
        self.bias = torch.nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        torch.nn.init.kaiming_uniform_(self.weight, a=math.sqrt(5))
        if self.bias is not None:
            bound = 1.0 / math.sqrt(self.in_channels)
            torch.nn.init.uniform_(self.bias, -bound, bound)

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)


class LayerNorm(torch.nn.Module):
    def __init__(self, in_channels, eps=1e-5, affine=True, mode="graph"):
        super().__init__()
        assert mode == "graph" and not affine
        self.in_channels, self.eps = in_channels, eps

    def forward(self, x, batch=None):
        if batch is None:
            x = x - x.mean()
            return x / (x.std(unbiased=False) + self.eps)
        b = int(batch.max()) + 1
        norm = degree(batch, b, dtype=x.dtype).clamp_(min=1).mul_(x.size(-1)).view(-1, 1)
        mean = scatter(x, batch, 0, dim_size=b, reduce="add").sum(dim=-1, keepdim=True) / norm
        x = x - mean.index_select(0, batch)
        var = scatter(x * x, batch, 0, dim_size=b, reduce="add").sum(dim=-1, keepdim=True) / norm
        return x / (var + self.eps).sqrt().index_select(0, batch)


class MessagePassing(torch.nn.Module):
    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2, **kwargs):
        super().__init__()
        self.aggr, self.node_dim = aggr, node_dim
        self._msg_args = [p for p in inspect.signature(self.message).parameters]

    def propagate(self, edge_index, size=None, **kwargs):
        src, dst = edge_index[0], edge_index[1]
        size_i = None
        args = {}
        for name in self._msg_args:
            if name.endswith("_i") and name[:-2] in kwargs:
                t = kwargs[name[:-2]]
                size_i = t.size(0)
                args[name] = t.index_select(0, dst)
            elif name.endswith("_j") and name[:-2] in kwargs:
                args[name] = kwargs[name[:-2]].index_select(0, src)
        for name in self._msg_args:
            if name in args:
                continue
            if name == "index":
                args[name] = dst
            elif name == "ptr":
                args[name] = None
            elif name == "size_i":
                args[name] = size_i
            else:
                args[name] = kwargs.get(name)
        msg = self.message(**args)
        return scatter(msg, dst, 0, dim_size=size_i, reduce="sum")


class SparseTensor:  # imported by sbftransformer_conv.py, never instantiated
    pass


def install():
    """Register the shim modules in ``sys.modules`` (idempotent)."""
    if "torch_geometric" in sys.modules and getattr(sys.modules["torch_geometric"], "_x2g_shim", False):
        return

    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        m._x2g_shim = True
        sys.modules[name] = m
        return m

    mod("torch_scatter", scatter_add=scatter_add, scatter_mean=scatter_mean, scatter=scatter)
    mod("torch_sparse", SparseTensor=SparseTensor)
    pyg = mod("torch_geometric")
    pyg.data = mod("torch_geometric.data", Data=Data)
    pyg.utils = mod("torch_geometric.utils", softmax=softmax, degree=degree,
                    remove_self_loops=remove_self_loops)
    pyg.typing = mod("torch_geometric.typing", Adj=object, OptTensor=object, PairTensor=object)
    pyg.loader = mod("torch_geometric.loader", DataLoader=None)
    nn = mod("torch_geometric.nn", LayerNorm=LayerNorm)
    pyg.nn = nn
    nn.conv = mod("torch_geometric.nn.conv", MessagePassing=MessagePassing)
    nn.dense = mod("torch_geometric.nn.dense")
    nn.dense.linear = mod("torch_geometric.nn.dense.linear", Linear=Linear)
