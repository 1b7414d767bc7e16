"""SBF-transformer trunk over the line graph (reference model.py:11-98), same module tree and
``forward(data, edge_index_0, atom_batch)`` surface.

Per layer: conv -> graph LayerNorm (per molecule) -> ResidualLayer -> SiLU(Linear) -> +residual
-> 2 x ResidualLayer -> readout; energies are the per-atom readouts summed over layers and
pooled per molecule.  Graph kernels (attention, LayerNorm, pools) run in libx2g.so; the dense
E- and N-row layers are fp32 GEMMs.

``data`` is the line-graph ``Data`` of the reference (x[E,D], edge_index[2,T], edge_attr,
batch[E], edge_sbf[T,42], node_rbf[E,R]).  Two additions let ``xgnn_poly`` skip work the
reference repeats per triplet: ``data._x2g_plan`` (a prebuilt :class:`GraphPlan`) and
``data.edge_attr_row`` — when present, ``edge_attr`` is a per-element table [10, D] and line
node e uses row ``edge_attr_row[e]``, so ``edgenn`` and every ``lin_edge`` run on 10 rows
instead of T (the reference's edge_attr rows are copies of those rows, xgnn.py:57-58).
"""
from __future__ import annotations

import torch
import torch.nn as nn
from torch.nn import ModuleList, Sequential, SiLU

from . import ops
from .layers import AtomWise, Linear, MolWise, ResidualLayer, run_mlp
from .plan import GraphPlan
from .sbftransformer_conv import SBFTransformerConv


class LayerNorm(nn.Module):
    """torch_geometric.nn.LayerNorm(mode='graph', affine=False) on contiguous molecule segments."""

    def __init__(self, in_channels, eps=1e-5, affine=False, mode="graph"):
        super().__init__()
        if affine or mode != "graph":
            raise NotImplementedError("graph mode, affine=False (X2-GNN's configuration)")
        self.in_channels, self.eps = in_channels, eps

    def forward(self, x, batch=None, rowptr=None, num_graphs=None):
        if rowptr is None and batch is None:
            xc = x - x.mean()
            return xc / (xc.std(unbiased=False) + self.eps)
        if rowptr is None:
            num_graphs = int(batch.max()) + 1
            rowptr = ops.csr_rowptr(batch, num_graphs)
        return ops.graph_layer_norm(x, rowptr, num_graphs, self.eps)


def _plan_of(data, edge_index_0, atom_batch):
    plan = data._store.get("_x2g_plan") if hasattr(data, "_store") else None
    return plan if plan is not None else GraphPlan.from_line_data(data, edge_index_0, atom_batch)


class _Trunk(nn.Module):
    def _build(self, conv_layers, emb_size, sbf_dim, rbf_dim, in_channels, heads, readout):
        self.in_channels = in_channels
        self.rbf_dim = rbf_dim
        self.edgenn = Sequential(Linear(emb_size, emb_size), SiLU(), Linear(emb_size, emb_size))
        self.convs = ModuleList([
            SBFTransformerConv(in_channels=in_channels, out_channels=int(in_channels / heads), heads=heads,
                               sbf_dim=sbf_dim * rbf_dim, rbf_dim=rbf_dim, dropout=0, edge_dim=emb_size)
            for _ in range(conv_layers)])
        self.readouts = ModuleList([readout() for _ in range(conv_layers + 1)])
        self.bf_skip = ModuleList([ResidualLayer(in_channels) for _ in range(conv_layers)])
        self.af_skip = ModuleList([Sequential(ResidualLayer(in_channels), ResidualLayer(in_channels))
                                   for _ in range(conv_layers)])
        self.dense_bf_skip = ModuleList([Linear(in_channels, in_channels, bias=True) for _ in range(conv_layers)])
        self.AF = SiLU()
        self.LayerNorm = LayerNorm(in_channels=in_channels, eps=1e-8, affine=False)
        self.conv_layers = conv_layers

    def edge_table_stages(self):
        """edgenn -> every conv's lin_edge as (Linear, act, parent) stages for ops.table_chain (parent
        -1 = the element table, 0 = edgenn's output), or None for another layout."""
        mods = list(self.edgenn)
        if len(mods) != 3 or not (isinstance(mods[0], Linear) and isinstance(mods[1], SiLU)
                                  and isinstance(mods[2], Linear)):
            return None
        if any(c.lin_edge is None for c in self.convs):
            return None
        return ([(mods[0], ops.ACT_SILU, -1), (mods[2], ops.ACT_NONE, 0)]
                + [(c.lin_edge, ops.ACT_NONE, 1) for c in self.convs])

    def _layers(self, data, plan, readout_fn, feature_fn=None, pool_fn=None, pool_out=None):
        """The conv layers with their readouts; ``pool_out = (seg_rowptr, S)``: the batched readout heads
        may sum the per-atom results per molecule themselves (the result then carries ``_x2g_pooled``)."""
        per_dst = "edge_attr_row" in data._store
        edge_proj = data._store.get("_x2g_edge_proj") if per_dst else None
        # lin_edge tables precomputed by the featurisation's table chain, or edgenn here
        edge_attr = run_mlp(self.edgenn, data.edge_attr) if edge_proj is None else None
        edge_row = data.edge_attr_row if per_dst else None
        out = data.x
        # The readouts (reference model.py:41,50) hang off the layer chain; results accumulate in
        # layer order (deterministic).  (Run on a second stream, overlapping the next layer, they
        # measured slower: 6.30 vs 6.00 ms/step — the persistent one-workgroup-per-CU kernels of the
        # main chain lose more to the shared CUs than the overlap gains; that path is gone.)
        results = None
        # Batched readout MLPs: collect every readout's MLP input, then one batched launch per MLP
        # layer for all readouts (ops.readout_mlps) instead of three launches per readout.
        grouped = out.is_cuda and feature_fn is not None
        feats = []
        # the readouts' edge -> atom pools of every layer output as one launch each way (pool_fn,
        # ops.rbf_pool_batch) after the last layer; per readout where that is unsupported
        pooled_xs = [] if grouped and pool_fn is not None else None

        def readout(i, x):
            nonlocal results
            if pooled_xs is not None:
                pooled_xs.append(x)
                return
            if grouped:
                feats.append(feature_fn(i, x))
                return
            r = readout_fn(i, x)
            results = r if results is None else results + r

        # gradient fan-in in place: the layer inputs and the radial basis feed several fused ops each
        fan = self._fan_in_ok(data, out)
        if fan:
            data.node_rbf._x2g_fanin = ops.FanIn()
            out._x2g_fanin = ops.FanIn()
        readout(0, out)
        sbf = data.edge_sbf
        # (every layer's S projected up front in one launch, x2g_sbf_project_batch, measured 1.2 % slower in
        # the step A/B, profiles/r4ab1_step_ab_sbatch_feat.log: each layer's S written right before its
        # attention is still in the MALL when the attention reads it; projected 3 layers early it is not)
        for i in range(self.conv_layers):
            res0 = out
            out = self.convs[i](sbf=sbf, rbf=data.node_rbf, x=out, edge_index=data._store.get("edge_index"),
                                edge_attr=edge_attr, line_graph=plan.lg, edge_row=edge_row,
                                edge_proj=edge_proj[i] if edge_proj is not None else None)
            stats = getattr(out, "_x2g_rowstats", None)
            if stats is not None and self._ln_fusable(out, i):
                # the LayerNorm runs inside the tail's row chain, from the conv's per-row statistics
                out = self._tail(i, out, res0, ln=(stats, plan.line_ptr, plan.num_graphs, self.LayerNorm.eps))
            else:
                out = self.LayerNorm(out, rowptr=plan.line_ptr, num_graphs=plan.num_graphs)
                out = self._tail(i, out, res0)
            if fan:
                out._x2g_fanin = ops.FanIn()
            readout(i + 1, out)
        if pooled_xs is not None:
            feats = pool_fn(pooled_xs)
            if feats is None:
                feats = [feature_fn(i, x) for i, x in enumerate(pooled_xs)]
        if grouped:
            mlps = [r.mlp for r in self.readouts]
            if ops.readout_mlps_supported(feats, mlps):
                r = ops.readout_mlps(feats, mlps, pool=pool_out)
                if pool_out is not None:
                    r._x2g_pooled = True
                return r
            for m, f in zip(mlps, feats):
                r = run_mlp(m, f)
                results = r if results is None else results + r
        return results


    def _pool_batch(self, xs, rbf, edge_index_0, plan):
        """Every readout's edge -> atom pool (readout.py:39-41 / 66-67) in one launch each way, or
        None where the batched kernels do not cover the shapes."""
        lins = [r.lin_rbf for r in self.readouts]
        if rbf is None or len(xs) != len(lins) or not ops.rbf_pool_batch_supported(xs, rbf, [l.weight for l in lins]):
            return None
        return ops.rbf_pool_batch(xs, rbf, [l.weight for l in lins], [l.bias for l in lins], edge_index_0,
                                  plan.atom_rowptr, plan.num_atoms)

    def _tail_linears(self, i):
        lins = [self.bf_skip[i].lin0, self.bf_skip[i].lin1, self.dense_bf_skip[i]]
        for r in self.af_skip[i]:
            lins += [r.lin0, r.lin1]
        return lins

    def _fan_in_ok(self, data, x):
        """True when every consumer of the layer inputs (readout rbf pool, conv projections, the
        tail's residual) and of the radial basis (readout pools, conv gates) is a fan-aware fused op,
        so their input gradients can be summed in place (ops.FanIn) instead of by autograd adds."""
        if not (ops._FAN_IN and x.is_cuda and x.dim() == 2 and torch.is_grad_enabled()):
            return False
        rbf = data.node_rbf
        if rbf is None or not ops.gate_supported(x.shape[1], rbf.shape[1]):
            return False
        for i, c in enumerate(self.convs):
            if not c.root_weight or not ops.conv_proj_fused_supported(
                    x, rbf, (c.lin_query.weight, c.lin_key.weight, c.lin_value.weight, c.lin_skip.weight),
                    (c.lin_query.bias, c.lin_key.bias, c.lin_value.bias, c.lin_skip.bias)):
                return False
            if not (ops._CHAIN and ops.chain_supported(x, self._tail_linears(i))):
                return False
        return True

    def _ln_fusable(self, x, i):
        """True when the graph LayerNorm before layer i's tail can run inside its row chain."""
        return ops._CHAIN and ops.chain_supported(x, self._tail_linears(i))

    def _tail(self, i, out, res0, ln=None):
        """bf_skip -> SiLU(dense_bf_skip(.)) + res0 -> af_skip (model.py:47-50): one row-chain
        kernel each way (ops.row_chain, 7 Linear stages) where compiled, else layer by layer.
        ``ln``: the row chain applies the preceding graph LayerNorm to ``out`` itself."""
        lins = self._tail_linears(i)
        if ops._CHAIN and ops.chain_supported(out, lins):
            S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
            flags = [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH]
            return ops.row_chain(out, res0, lins, flags, ln=ln)
        out = self.bf_skip[i](out)
        out = self.dense_bf_skip[i].fused(out, act=ops.ACT_SILU, res=res0)  # SiLU(dense(out)) + res0
        return self.af_skip[i](out)


class SBFTransformer(_Trunk):
    """Trunk with per-atom readouts (extensive targets, reference model.py:11-54)."""

    def __init__(self, conv_layers, emb_size, sbf_dim, rbf_dim=16, in_channels=128, heads=8):
        super().__init__()
        self._build(conv_layers, emb_size, sbf_dim, rbf_dim, in_channels, heads,
                    lambda: AtomWise(in_channels=in_channels, rbf_dim=rbf_dim, num_target=1))

    def forward(self, data, edge_index_0, atom_batch):
        plan = _plan_of(data, edge_index_0, atom_batch)

        def readout(i, x):
            return self.readouts[i](x=x, rbf=data.node_rbf, num_atoms=plan.num_atoms, edge_index_0=edge_index_0,
                                    atom_rowptr=plan.atom_rowptr)

        def features(i, x):
            return self.readouts[i].features(x=x, rbf=data.node_rbf, num_atoms=plan.num_atoms,
                                             edge_index_0=edge_index_0, atom_rowptr=plan.atom_rowptr)

        def pools(xs):
            return self._pool_batch(xs, data.node_rbf, edge_index_0, plan)

        # the global add pool (model.py:53) fused into the batched readout heads where they run
        pool_out = (plan.mol_ptr, plan.out_graphs) if plan.out_graphs == plan.num_graphs else None
        per_atom = self._layers(data, plan, readout, features, pools, pool_out=pool_out)
        if getattr(per_atom, "_x2g_pooled", False):
            return per_atom.view(-1)
        return ops.segment_sum(per_atom, plan.mol_ptr, plan.out_graphs).view(-1)


class SBFTransformerGlobal(_Trunk):
    """Trunk with per-molecule readouts (intensive targets, reference model.py:56-98)."""

    def __init__(self, conv_layers, emb_size, sbf_dim, rbf_dim=16, in_channels=128, heads=8, pool_option="mean"):
        super().__init__()
        self._build(conv_layers, emb_size, sbf_dim, rbf_dim, in_channels, heads,
                    lambda: MolWise(in_channels=in_channels, rbf_dim=rbf_dim, num_target=1, pool_option=pool_option))

    def forward(self, data, edge_index_0, atom_batch):
        plan = _plan_of(data, edge_index_0, atom_batch)

        kw = dict(rbf=data.node_rbf, num_atoms=plan.num_atoms, edge_index_0=edge_index_0, atom_batch=atom_batch,
                  dim_size=plan.out_graphs, atom_rowptr=plan.atom_rowptr, mol_rowptr=plan.mol_ptr[: plan.out_graphs + 1])

        def readout(i, x):
            return self.readouts[i](x=x, **kw)

        def features(i, x):
            return self.readouts[i].features(x=x, **kw)

        def pools(xs):
            atoms = self._pool_batch(xs, data.node_rbf, edge_index_0, plan)
            if atoms is None:
                return None
            return [r.finish(a, atom_batch, plan.out_graphs, kw["mol_rowptr"]) for r, a in zip(self.readouts, atoms)]

        return self._layers(data, plan, readout, features, pools).view(-1)
