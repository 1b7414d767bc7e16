"""Test infrastructure: import the reference (``/root/reference``, read-only) in THIS container.

Used only by ``make_golden.py`` to produce the committed fixtures; nothing on the GPU box or in
the product imports it.  The reference files are not modified; the harness applies the four
run-time patches SURVEY.md §8(c) lists for the reference's defects in this environment:

1. restated PyG / torch_scatter modules (``pyg_shim.install``);
2. ``np.math = math`` (basis_func.py:174 uses ``np.math.factorial``, gone in numpy 2);
3. ``torch.nn.init.zeros`` (sbftransformer_conv.py:81-82 calls it; it does not exist, and
   ``lin_rbf.bias`` is None);
4. ``edge_graph.sp`` wrapped so scipy sparse matrices accept torch index keys
   (edge_graph.py:15-27; scipy 1.15 rejects torch tensors as indices).

``sys.dont_write_bytecode`` keeps ``__pycache__`` out of the reference tree.
"""
from __future__ import annotations

import math
import os
import sys
import types

import numpy as np
import scipy.sparse as sps
import torch

REF = "/root/reference"


def _np(key):
    if torch.is_tensor(key):
        return key.numpy()
    if isinstance(key, tuple):
        return tuple(_np(k) for k in key)
    return key


class _CSR(sps.csr_matrix):
    def __getitem__(self, key):
        return super().__getitem__(_np(key))


class _COO:
    def __init__(self, arg, shape=None):
        data, ij = arg
        self._m = sps.coo_matrix((np.asarray(_np(data)), (np.asarray(_np(ij[0])), np.asarray(_np(ij[1])))),
                                 shape=shape)

    def tocsr(self):
        return _CSR(self._m.tocsr())


def import_reference():
    """Return a namespace with the reference modules (xgnn, model, sbftransformer_conv, ...)."""
    if not os.path.isdir(REF):
        raise RuntimeError("reference tree not present (fixture generation runs only in the build container)")
    sys.dont_write_bytecode = True
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import pyg_shim  # noqa: E402

    pyg_shim.install()
    np.math = math
    if not hasattr(torch.nn.init, "zeros"):
        torch.nn.init.zeros = lambda t: None if t is None else t.zero_()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import edge_graph  # noqa: E402

    edge_graph.sp = types.SimpleNamespace(coo_matrix=_COO)
    import angular_basis_layer, atom_embedding, envelop, model, radial_basis_layer  # noqa: E401,E402
    import readout, residual_layer, sbftransformer_conv, xgnn  # noqa: E401,E402

    return types.SimpleNamespace(
        xgnn=xgnn, model=model, sbftransformer_conv=sbftransformer_conv, edge_graph=edge_graph,
        angular_basis_layer=angular_basis_layer, radial_basis_layer=radial_basis_layer,
        envelop=envelop, atom_embedding=atom_embedding, readout=readout, residual_layer=residual_layer,
    )
