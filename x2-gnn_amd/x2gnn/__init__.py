"""x2gnn — MI355X-native X2-GNN message-passing hot path.

Host side (this package): the reference's model / operator surface (``xgnn_poly``,
``SBFTransformer``, ``SBFTransformerConv``, PyG-style ``Data``/``Batch``) on PyTorch-ROCm.
Device side: ``libx2g.so`` (hand-written gfx950 HIP kernels behind the C ABI in
``include/x2g.h``), loaded through :mod:`x2gnn._lib`.
"""
from .data import Batch, Data, collate, molecule_to_data
from .layers import AtomWise, EmbeddingBlock, F_B_2D, MolWise, RadialBasis, ResidualLayer, poly_envelop
from .model import LayerNorm, SBFTransformer, SBFTransformerGlobal
from .plan import GraphPlan
from .sbftransformer_conv import SBFTransformerConv
from .xgnn import xgnn_poly, xgnn_poly_global

__all__ = [
    "AtomWise", "Batch", "Data", "EmbeddingBlock", "F_B_2D", "GraphPlan", "LayerNorm", "MolWise", "RadialBasis",
    "ResidualLayer", "SBFTransformer", "SBFTransformerConv", "SBFTransformerGlobal", "collate", "molecule_to_data",
    "poly_envelop", "xgnn_poly", "xgnn_poly_global",
]
