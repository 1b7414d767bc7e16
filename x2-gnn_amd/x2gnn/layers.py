"""Featurisation and readout blocks of X2-GNN with the reference's constructor arguments and
parameter names (so reference ``state_dict``s load unchanged).

================  =======================================  ==========================================
class             reference                                 device path here
================  =======================================  ==========================================
poly_envelop      envelop.py:5-21                           fused into x2g_edge_basis
RadialBasis       radial_basis_layer.py:26-40 (trainable)   x2g_edge_basis (+ its frequency gradient)
F_B_2D            angular_basis_layer.py:51-93 (+sympy)      x2g_bessel_env + x2g_spherical_basis;
                                                            constants precomputed, no sympy at run time
EmbeddingBlock    atom_embedding.py:10-25                    per-element table (x2g_embedding_table)
ResidualLayer     residual_layer.py:5-27                     fused f32-MFMA dense kernels (the trunk's
                                                            seven tail layers: one row-chain kernel)
AtomWise          readout.py:7-43                            x2g_rbf_pool (lin_rbf gate + pool fused) or
                                                            lin_rbf + x2g_segment_sum(x * rf); MLP fused
MolWise           readout.py:45-76                           + segment sum/mean over molecules
================  =======================================  ==========================================
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


class Linear(nn.Linear):
    """nn.Linear (same parameters / state_dict keys) running the fused dense kernels.

    ``fused(x, act, res)`` = act(x W^T + b) + res in one kernel.  On CPU tensors it is plain
    nn.Linear math so modules can be built, loaded and inspected on the host."""

    def forward(self, x):
        return self.fused(x)

    def fused(self, x, act=ops.ACT_NONE, res=None):
        if x.is_cuda:
            return ops.dense(x, self.weight, self.bias, act=act, res=res)
        y = super().forward(x)
        if act == ops.ACT_SILU:
            y = F.silu(y)
        return y if res is None else y + res


def run_mlp(layers, x):
    """Apply a [Linear, SiLU, ..., Linear] stack, fusing each Linear with the SiLU after it."""
    mods = list(layers)
    i = 0
    while i < len(mods):
        m = mods[i]
        if isinstance(m, Linear) and i + 1 < len(mods) and isinstance(mods[i + 1], nn.SiLU):
            x = m.fused(x, act=ops.ACT_SILU)
            i += 2
        else:
            x = m(x)
            i += 1
    return x


class poly_envelop(nn.Module):
    """u(d) = 1/x + a x^(p-1) + b x^p + c x^(p+1), x = d/cutoff, p = exponent+1 (no cutoff mask)."""

    def __init__(self, cutoff, exponent):
        super().__init__()
        self.inv_cutoff = 1.0 / cutoff
        self.exponent = exponent
        self.p = exponent + 1
        p = self.p
        self.a, self.b, self.c = -(p + 1) * (p + 2) / 2, p * (p + 2), -p * (p + 1) / 2

    def forward(self, distances):
        x = distances * self.inv_cutoff
        xp = x ** (self.p - 1)
        return 1.0 / x + self.a * xp + self.b * (xp * x) + self.c * (xp * x * x)


class RadialBasis(nn.Module):
    """sin(f_n d / cutoff), f_n initialised to n*pi and trainable (the ``frequencies`` parameter)."""

    def __init__(self, embedding_size, cutoff, Trainable=True, **kwargs):
        super().__init__(**kwargs)
        self.num_radial = embedding_size
        self.inv_cutoff = 1.0 / cutoff
        f = math.pi * torch.arange(1, embedding_size + 1, dtype=torch.float32)
        if Trainable:
            self.frequencies = nn.Parameter(f)
        else:
            self.register_buffer("frequencies", f)

    def forward(self, bond_distances):
        return torch.sin(self.frequencies * (bond_distances * self.inv_cutoff).unsqueeze(-1))


class F_B_2D(nn.Module):
    """Spherical-Bessel x Y_l0 basis, [T, num_spherical*num_radial], l-major columns.

    Compiled for num_spherical <= 7 and num_radial <= 16 (config.json: 7 x 6; the reference's
    default xgnn_poly: 7 x 16, xgnn.py:16) with envelope exponent 5; the expanded formulas'
    coefficients come from scripts/gen_basis_consts.py (no sympy at run time).
    """

    def __init__(self, num_spherical, num_radial, cutoff, envelope_exponent=5):
        super().__init__()
        if not (1 <= num_spherical <= 7 and 1 <= num_radial <= 16) or envelope_exponent != 5:
            raise NotImplementedError("compiled basis: num_spherical <= 7, num_radial <= 16, envelope exponent 5")
        self.num_spherical, self.num_radial, self.cutoff = num_spherical, num_radial, cutoff

    def radial(self, d):
        """[E, S] env(d) * N_ln j_l(z_ln d / cutoff) (the E-row half of the reference forward)."""
        return ops.bessel_env(d, self.cutoff, self.num_spherical, self.num_radial)

    def forward(self, d, Angles, edge_index_1):
        return ops.spherical_basis_from_angles(Angles, edge_index_1, self.radial(d), self.num_spherical,
                                               self.num_radial)

    def from_positions(self, d, pos, line_graph, radial=None, lazy=False):
        """Fast path: angles computed in-kernel from the triplets' atom positions (xgnn.py:61-65);
        ``radial`` = precomputed ``self.radial(d)`` (x2g_edge_basis writes it); ``lazy``: the [T, S] rows
        are filled only if a consumer reads them (ops.materialize_sbf)."""
        return ops.spherical_basis(pos, line_graph, self.radial(d) if radial is None else radial,
                                   num_spherical=self.num_spherical, num_radial=self.num_radial, lazy=lazy)


class _ScaleGradByCount(torch.autograd.Function):
    """Identity on the embedding table; backward divides row z by its count (scale_grad_by_freq)
    and zeroes the padding row, as ATen's embedding backward does."""

    @staticmethod
    def forward(ctx, weight, counts, padding_idx):
        ctx.save_for_backward(counts)
        ctx.padding_idx = padding_idx
        # a copy, not a view: the renorm mutates the weight in place on the next forward
        return weight.clone()

    @staticmethod
    def backward(ctx, g):
        (counts,) = ctx.saved_tensors
        g = g / counts.clamp(min=1).to(g.dtype).unsqueeze(1)
        if ctx.padding_idx is not None:
            g = g.clone()
            g[ctx.padding_idx] = 0
        return g, None, None


class EmbeddingBlock(nn.Module):
    """SiLU(Linear(Embedding(Z))) with Embedding(10, D, padding_idx=0, max_norm=3, scale_grad_by_freq)."""

    def __init__(self, embedding_size=128, activation=True, **kwargs):
        super().__init__(**kwargs)
        self.AF = nn.SiLU()
        self.embedding = nn.Embedding(10, embedding_size, padding_idx=0, max_norm=3.0, scale_grad_by_freq=True)
        self.lin = Linear(embedding_size, embedding_size, bias=True)
        self.activate = activation

    def forward(self, atomic_num):
        return self.lin.fused(self.embedding(atomic_num), act=ops.ACT_SILU if self.activate else ops.ACT_NONE)

    def element_rows(self, atomic_num, count_z=None):
        """The embedding rows [num_embeddings, D] the Linear of ``element_table`` reads (renormalised
        as the embedding lookup does), from one launch (csrc/embedding.hip); None where that kernel
        does not apply (CPU, other norms, large vocabularies).  ``count_z``: the atomic numbers the
        per-batch rules (renormalised rows, scale_grad_by_freq counts) are evaluated over, when not
        ``atomic_num`` itself (a molecule shard of a global batch, dist.collate_shard)."""
        emb = self.embedding
        z = (atomic_num if count_z is None else count_z).reshape(-1)
        if z.is_cuda and emb.norm_type == 2.0 and emb.num_embeddings <= 64:
            return ops.embedding_table(emb.weight, z, emb.max_norm, emb.padding_idx, emb.scale_grad_by_freq)
        return None

    def element_table(self, atomic_num, count_z=None):
        """Per-element rows [num_embeddings, D] equal to forward(z) for every z present.

        Reproduces the in-place max_norm renormalisation of the rows referenced by
        ``atomic_num`` (torch.embedding_renorm_) and the scale_grad_by_freq gradient, without
        materialising the [N, D] output: row z of the result stands for every atom of type z.
        """
        emb = self.embedding
        z = (atomic_num if count_z is None else count_z).reshape(-1)
        w = self.element_rows(atomic_num, count_z)
        if w is not None:
            return self.lin.fused(w, act=ops.ACT_SILU if self.activate else ops.ACT_NONE)
        # counts per element without torch.bincount (its output size is data-dependent: a host sync
        # that would also break HIP-graph capture); float counts are exact below 2^24
        counts = torch.zeros(emb.num_embeddings, dtype=torch.float32, device=z.device)
        counts.index_add_(0, z, torch.ones(z.shape[0], dtype=torch.float32, device=z.device))
        w = emb.weight
        if emb.max_norm is not None:
            with torch.no_grad():
                norms = w.norm(p=emb.norm_type, dim=1)
                scale = torch.where((counts > 0) & (norms > emb.max_norm), emb.max_norm / (norms + 1e-7),
                                    torch.ones_like(norms))
                w.mul_(scale.unsqueeze(1))
        if emb.scale_grad_by_freq or emb.padding_idx is not None:
            c = counts if emb.scale_grad_by_freq else torch.ones_like(counts)
            w = _ScaleGradByCount.apply(w, c, emb.padding_idx)
        return self.lin.fused(w, act=ops.ACT_SILU if self.activate else ops.ACT_NONE)


class ResidualLayer(nn.Module):
    """x + SiLU(lin1(SiLU(lin0(x))))."""

    def __init__(self, in_channels, bias=True):
        super().__init__()
        self.lin0 = Linear(in_channels, in_channels, bias=bias)
        self.lin1 = Linear(in_channels, in_channels, bias=bias)
        self.AF = nn.SiLU()

    def forward(self, x):
        if x.is_cuda:  # both dense kernels + a backward that folds the residual into dx
            return ops.residual_layer(x, self.lin0.weight, self.lin0.bias, self.lin1.weight, self.lin1.bias)
        h = self.lin0.fused(x, act=ops.ACT_SILU)
        return self.lin1.fused(h, act=ops.ACT_SILU, res=x)


def _mlp(in_channels, num_target, depth):
    layers = []
    for _ in range(depth - 1):
        layers += [Linear(in_channels, in_channels), nn.SiLU()]
    layers.append(Linear(in_channels, num_target))
    return nn.ModuleList(layers)


def _edge_pool(x, rbf, lin_rbf, edge_index_0, num_atoms, atom_rowptr):
    """sum over edges e with source atom n of lin_rbf(rbf)[e] * x[e] -> [num_atoms, D]."""
    if atom_rowptr is None:
        atom_rowptr = ops.csr_rowptr(edge_index_0, num_atoms)
    if ops.gate_supported(x.shape[1], rbf.shape[1]):  # the [E, D] filter is never materialised
        return ops.rbf_pool(x, rbf, lin_rbf.weight, lin_rbf.bias, edge_index_0, atom_rowptr, num_atoms)
    return ops.segment_sum(x, atom_rowptr, num_atoms, mul=lin_rbf(rbf))


class AtomWise(nn.Module):
    """Per-atom readout: (lin_rbf(rbf) * x) pooled edges->atoms by source atom, then an MLP."""

    def __init__(self, mlp_depth=3, in_channels=256, rbf_dim=16, num_target=1):
        super().__init__()
        self.mlp = _mlp(in_channels, num_target, mlp_depth)
        self.lin_rbf = Linear(rbf_dim, in_channels)

    def features(self, x, rbf, num_atoms, edge_index_0, atom_rowptr=None):
        """The MLP input (everything before readout.py:42's MLP)."""
        return _edge_pool(x, rbf, self.lin_rbf, edge_index_0, num_atoms, atom_rowptr)

    def forward(self, x, rbf, num_atoms, edge_index_0, atom_rowptr=None):
        return run_mlp(self.mlp, self.features(x, rbf, num_atoms, edge_index_0, atom_rowptr))


class MolWise(nn.Module):
    """Per-molecule readout: edges->atoms pool, atoms->molecules mean/add pool, then an MLP."""

    def __init__(self, mlp_depth=3, in_channels=256, rbf_dim=6, num_target=1, pool_option="mean"):
        super().__init__()
        if pool_option not in ("mean", "add"):
            raise AssertionError("unsupport pooling option")
        self.lin_rbf = Linear(rbf_dim, in_channels)
        self.mlp = _mlp(in_channels, num_target, mlp_depth)
        self.pool_option = pool_option

    def features(self, x, rbf, num_atoms, edge_index_0, atom_batch, dim_size, atom_rowptr=None, mol_rowptr=None):
        """The MLP input: edges -> atoms -> molecules (readout.py:66-71)."""
        out = _edge_pool(x, rbf, self.lin_rbf, edge_index_0, num_atoms, atom_rowptr)
        return self.finish(out, atom_batch, dim_size, mol_rowptr)

    def finish(self, out, atom_batch, dim_size, mol_rowptr=None):
        """atoms -> molecules (readout.py:68-71) of the pooled [num_atoms, D] features."""
        if mol_rowptr is None:
            mol_rowptr = ops.csr_rowptr(atom_batch, dim_size)
        pooled = ops.segment_sum(out, mol_rowptr, dim_size)
        if self.pool_option == "mean":
            cnt = (mol_rowptr[1:] - mol_rowptr[:-1]).clamp(min=1).to(pooled.dtype)
            pooled = pooled / cnt.unsqueeze(1)
        return pooled

    def forward(self, x, rbf, num_atoms, edge_index_0, atom_batch, dim_size, atom_rowptr=None, mol_rowptr=None):
        return run_mlp(self.mlp, self.features(x, rbf, num_atoms, edge_index_0, atom_batch, dim_size, atom_rowptr,
                                               mol_rowptr))
