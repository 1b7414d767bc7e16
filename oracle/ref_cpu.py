"""Oracle (test infrastructure): torch-CPU fp32 restatement of X2-GNN's forward.

Op-for-op with the reference (file:line cited per block) and with PyG 2.1.0 / torch_scatter
2.1.0 operator semantics restated:

* MessagePassing.propagate (aggr='add'): ``x_i = x.index_select(0, edge_index[1])``,
  ``x_j = x.index_select(0, edge_index[0])``, message, ``scatter(..., reduce='sum')``;
* utils.softmax: subtract the segment max, exp, divide by (segment sum + 1e-16);
* nn.LayerNorm(mode='graph'): per-graph mean/var over rows x channels, x / sqrt(var + eps);
* scatter_add / scatter_mean: ``index_add_`` into ``dim_size`` rows (deterministic on CPU).

The module tree and parameter names equal the reference's, so the same seeded weights and
gradient keys apply.  The spherical Bessel functions are evaluated with scipy in float64 (the
reference evaluates sympy-expanded fp32 expressions that lose accuracy at small d; energies
move by < 2e-6).  Not imported by the product; used by tests and bench.py's
cpu_baseline.
"""
from __future__ import annotations

import functools
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from scipy import special
from scipy.optimize import brentq

from .triplets import vertex_to_edge

NUM_SPH, NUM_RAD = 7, 6  # config.json; the reference's own defaults are (7, 16) (xgnn.py:16)


# ------------------------------------------------------------------ basis constants (basis_func.py)
def _sph_jn(r, n):
    return np.sqrt(np.pi / (2 * r)) * special.jv(n + 0.5, r)


def _bessel_zeros(n, k):
    """basis_func.py:14-29: zeros bracketed from the previous order, stored as float32."""
    z = np.zeros((n, k), np.float32)
    z[0] = np.arange(1, k + 1) * np.pi
    pts = np.arange(1, k + n) * np.pi
    for i in range(1, n):
        r = np.array([brentq(_sph_jn, pts[j], pts[j + 1], (i,)) for j in range(k + n - 1 - i)], np.float32)
        z[i] = r[:k]
        pts = r
    return z


@functools.lru_cache(maxsize=None)
def _basis_consts(nsph, nrad):
    """(zeros [nsph, nrad] float64 of the float32 roots, normalisers N_ln) for F_B_2D(nsph, nrad)."""
    zeros = _bessel_zeros(nsph, nrad).astype(np.float64)
    norm = np.array([[1.0 / math.sqrt(0.5 * _sph_jn(zeros[l, n], l + 1) ** 2) for n in range(nrad)]
                     for l in range(nsph)])
    return zeros, norm


def bessel_radial(d_scaled: np.ndarray, nsph=NUM_SPH, nrad=NUM_RAD) -> np.ndarray:
    """[E, nsph * nrad] N_ln j_l(z_ln x), l-major (basis_func.py:47-71)."""
    zeros, norm = _basis_consts(nsph, nrad)
    x = np.asarray(d_scaled, np.float64)
    cols = []
    for l in range(nsph):
        for n in range(nrad):
            cols.append(norm[l, n] * special.spherical_jn(l, zeros[l, n] * x))
    return np.stack(cols, axis=1)


def sph_y0(theta: np.ndarray, nsph=NUM_SPH) -> np.ndarray:
    """[T, nsph] sqrt((2l+1)/4pi) P_l(cos theta) (basis_func.py:110-155, m = 0)."""
    c = np.cos(np.asarray(theta, np.float64))
    return np.stack([math.sqrt((2 * l + 1) / (4 * math.pi)) * special.eval_legendre(l, c) for l in range(nsph)],
                    axis=1)


def envelope(d, cutoff=5.0, exponent=5):
    """envelop.py:16-21."""
    p = exponent + 1
    a, b, c = -(p + 1) * (p + 2) / 2, p * (p + 2), -p * (p + 1) / 2
    x = d * (1 / cutoff)
    return 1 / x + a * x ** (p - 1) + b * x ** p + c * x ** (p + 1)


def spherical_basis(d, theta, jk, nsph=NUM_SPH, nrad=NUM_RAD):
    """F_B_2D(nsph, nrad).forward (angular_basis_layer.py:80-93) -> [T, nsph * nrad] float32."""
    rbf = bessel_radial(d.detach().numpy() / 5.0, nsph, nrad)
    env = envelope(d.detach().double()).numpy()
    rbf_env = env[:, None] * rbf
    cbf = np.repeat(sph_y0(theta.detach().numpy(), nsph), nrad, axis=1)
    return torch.from_numpy((rbf_env[jk.numpy()] * cbf).astype(np.float32))


# ------------------------------------------------------------------ restated PyG / torch_scatter
def scatter_sum(src, index, dim_size):
    out = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype)
    return out.index_add(0, index, src)


def scatter_max(src, index, dim_size):
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    out = torch.zeros((dim_size,) + tuple(src.shape[1:]), dtype=src.dtype)
    return out.scatter_reduce(0, idx, src, reduce="amax", include_self=False)


def pyg_softmax(src, index, num_nodes):
    mx = scatter_max(src, index, num_nodes).index_select(0, index)
    ex = (src - mx).exp()
    return ex / (scatter_sum(ex, index, num_nodes).index_select(0, index) + 1e-16)


def graph_layer_norm(x, batch, eps):
    b = int(batch.max()) + 1
    cnt = scatter_sum(torch.ones(batch.shape[0]), batch, b).clamp(min=1) * x.shape[1]
    mean = scatter_sum(x, batch, b).sum(-1, keepdim=True) / cnt.unsqueeze(1)
    xc = x - mean.index_select(0, batch)
    var = scatter_sum(xc * xc, batch, b).sum(-1, keepdim=True) / cnt.unsqueeze(1)
    return xc / (var + eps).sqrt().index_select(0, batch)


# ------------------------------------------------------------------ modules (same names as the reference)
class ResidualLayer(nn.Module):  # residual_layer.py:5-27
    def __init__(self, c):
        super().__init__()
        self.lin0, self.lin1, self.AF = nn.Linear(c, c), nn.Linear(c, c), nn.SiLU()

    def forward(self, x):
        return self.AF(self.lin1(self.AF(self.lin0(x)))) + x


class AtomWise(nn.Module):  # readout.py:7-43
    def __init__(self, c, rbf_dim, depth=3):
        super().__init__()
        layers = []
        for _ in range(depth - 1):
            layers += [nn.Linear(c, c), nn.SiLU()]
        self.mlp = nn.ModuleList(layers + [nn.Linear(c, 1)])
        self.lin_rbf = nn.Linear(rbf_dim, c)

    def pool(self, x, rbf, num_atoms, ei0):
        return scatter_sum(self.lin_rbf(rbf) * x, ei0, num_atoms)

    def forward(self, x, rbf, num_atoms, ei0, **_):
        out = self.pool(x, rbf, num_atoms, ei0)
        for layer in self.mlp:
            out = layer(out)
        return out


class MolWise(AtomWise):  # readout.py:45-76 (lin_rbf registered first there)
    def __init__(self, c, rbf_dim, depth=3, pool_option="mean"):
        nn.Module.__init__(self)
        self.lin_rbf = nn.Linear(rbf_dim, c)
        layers = []
        for _ in range(depth - 1):
            layers += [nn.Linear(c, c), nn.SiLU()]
        self.mlp = nn.ModuleList(layers + [nn.Linear(c, 1)])
        self.pool_option = pool_option

    def forward(self, x, rbf, num_atoms, ei0, atom_batch=None, dim_size=None):
        out = self.pool(x, rbf, num_atoms, ei0)
        s = scatter_sum(out, atom_batch, dim_size)
        if self.pool_option == "mean":
            s = s / scatter_sum(torch.ones(atom_batch.shape[0]), atom_batch, dim_size).clamp(min=1).unsqueeze(1)
        out = s
        for layer in self.mlp:
            out = layer(out)
        return out


class SBFTransformerConv(nn.Module):  # sbftransformer_conv.py:16-166
    def __init__(self, c, heads, sbf_dim, rbf_dim, edge_dim):
        super().__init__()
        self.heads, self.out_channels = heads, c // heads
        self.lin_key, self.lin_query, self.lin_value = nn.Linear(c, c), nn.Linear(c, c), nn.Linear(c, c)
        self.lin_edge = nn.Linear(edge_dim, c, bias=False)
        self.lin_skip = nn.Linear(c, c)
        self.lin_sbf = nn.Linear(sbf_dim, c)
        self.lin_rbf = nn.Linear(rbf_dim, c, bias=False)

    def forward(self, sbf, rbf, x, edge_index, edge_attr):
        H, C = self.heads, self.out_channels
        x_src = x * self.lin_rbf(rbf)                                        # :99-100
        q = self.lin_query(x).view(-1, H, C)                                # :105-107
        k = self.lin_key(x_src).view(-1, H, C)
        v = self.lin_value(x_src).view(-1, H, C)
        src, dst = edge_index[0], edge_index[1]
        q_i, k_j, v_j = q.index_select(0, dst), k.index_select(0, src), v.index_select(0, src)
        e = self.lin_edge(edge_attr).view(-1, H, C)                         # :144
        k_j = k_j + e
        s = self.lin_sbf(sbf)                                               # :148
        alpha = (q_i * k_j).sum(-1) / math.sqrt(C)                          # :150
        alpha = pyg_softmax(alpha, dst, x.shape[0])                         # :151
        msg = (v_j + e) * s.view(-1, H, C) * alpha.view(-1, H, 1)           # :155-160
        out = scatter_sum(msg, dst, x.shape[0]).view(-1, H * C)             # aggr='add'
        return out + self.lin_skip(x)                                       # :127


class Trunk(nn.Module):  # model.py:11-98
    def __init__(self, L, emb, sbf_dim, rbf_dim, c, heads, global_pool=None):
        super().__init__()
        self.edgenn = nn.Sequential(nn.Linear(emb, emb), nn.SiLU(), nn.Linear(emb, emb))
        self.convs = nn.ModuleList([SBFTransformerConv(c, heads, sbf_dim * rbf_dim, rbf_dim, emb) for _ in range(L)])
        if global_pool is None:
            self.readouts = nn.ModuleList([AtomWise(c, rbf_dim) for _ in range(L + 1)])
        else:
            self.readouts = nn.ModuleList([MolWise(c, rbf_dim, pool_option=global_pool) for _ in range(L + 1)])
        self.bf_skip = nn.ModuleList([ResidualLayer(c) for _ in range(L)])
        self.af_skip = nn.ModuleList([nn.Sequential(ResidualLayer(c), ResidualLayer(c)) for _ in range(L)])
        self.dense_bf_skip = nn.ModuleList([nn.Linear(c, c) for _ in range(L)])
        self.AF = nn.SiLU()
        self.global_pool = global_pool

    def forward(self, x, edge_index, edge_attr, batch, sbf, rbf, ei0, atom_batch):
        edge_attr = self.edgenn(edge_attr)                                   # model.py:39
        n_atoms = atom_batch.shape[0]
        b = int(batch.max()) + 1
        kw = dict(atom_batch=atom_batch, dim_size=b) if self.global_pool else {}
        out = x
        results = self.readouts[0](out, rbf, n_atoms, ei0, **kw)
        for i, conv in enumerate(self.convs):                                # model.py:43-51
            res0 = out
            out = conv(sbf, rbf, out, edge_index, edge_attr)
            out = graph_layer_norm(out, batch, 1e-8)
            out = self.bf_skip[i](out)
            out = self.AF(self.dense_bf_skip[i](out))
            out = out + res0
            out = self.af_skip[i](out)
            results = results + self.readouts[i + 1](out, rbf, n_atoms, ei0, **kw)
        if self.global_pool:
            return results.view(-1)
        return scatter_sum(results, atom_batch, b).view(-1)                  # model.py:53


class EmbeddingBlock(nn.Module):  # atom_embedding.py:10-25
    def __init__(self, d):
        super().__init__()
        self.AF = nn.SiLU()
        self.embedding = nn.Embedding(10, d, padding_idx=0, max_norm=3.0, scale_grad_by_freq=True)
        self.lin = nn.Linear(d, d)

    def forward(self, z):
        return self.AF(self.lin(self.embedding(z)))


class RadialBasis(nn.Module):  # radial_basis_layer.py:26-40
    def __init__(self, n):
        super().__init__()
        self.frequencies = nn.Parameter(math.pi * torch.arange(1, n + 1, dtype=torch.float32))

    def forward(self, d):
        return torch.sin(self.frequencies * (d * (1 / 5.0)).unsqueeze(-1))


class XGNN(nn.Module):  # xgnn.py:15-137
    def __init__(self, conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128,
                 global_pool=None):
        super().__init__()
        self.num_spherical, self.num_radial = sbf_dim, rbf_dim  # F_B_2D(sbf_dim, rbf_dim) (xgnn.py:34)
        self.AF = nn.SiLU()
        self.emb_block = EmbeddingBlock(embedding_size)
        self.rbf_layer = RadialBasis(rbf_dim)
        self.fin_model = Trunk(conv_layers, embedding_size, sbf_dim, rbf_dim, in_channels, heads, global_pool)
        self.mat_trans = nn.Linear(338, 2 * embedding_size)
        self.rbf_trans = nn.Linear(rbf_dim, embedding_size)
        self.emb_trans = nn.Linear(2 * embedding_size, in_channels)

    def forward(self, x, edge_index, edge_attr, atom_pos, edge_num, atom_batch):
        n = x.shape[0]
        d = torch.norm(atom_pos[edge_index[0]] - atom_pos[edge_index[1]], dim=1)        # :39
        batch = torch.arange(edge_num.shape[0]).repeat_interleave(edge_num)              # :44
        env = envelope(d)[:, None]                                                       # :49-50
        trip, j, i, k = (torch.from_numpy(a) for a in vertex_to_edge(edge_index.numpy(), n))  # :52
        neo_x = self.AF(self.mat_trans(edge_attr * env))                                 # :54-55
        neo_edge_attr = self.emb_block(x)[j]                                             # :57-58
        ji = atom_pos[i] - atom_pos[j]
        jk = atom_pos[k] - atom_pos[j]
        theta = torch.atan2(torch.norm(torch.cross(ji, jk, dim=1), dim=1), (ji * jk).sum(1))  # :61-64
        sbf = spherical_basis(d, theta, trip[0], self.num_spherical, self.num_radial)   # :65
        rbf = self.rbf_layer(d) * env                                                    # :68-69
        neo_x = self.AF(self.emb_trans(neo_x))                                           # :70
        return self.fin_model(neo_x, trip, neo_edge_attr, batch, sbf, rbf, edge_index[0], atom_batch)


def run_batch(model: XGNN, b):
    """Forward an x2gnn-style collated batch (CPU tensors)."""
    return model(b.x, b.edge_index, b.edge_attr, b.atom_pos, b.edge_num, b.batch)
