"""ORACLE — test infrastructure only.

A CPU restatement of zfwangDP/X2-GNN's message-passing hot path, used to check the gfx950
product path and as the ``cpu_baseline`` leg of bench.py.  Nothing in the product
(``x2-gnn_amd/``) imports, links or executes this package; only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline may.

Parity is PINNED: the restatement is checked against golden fixtures produced by running the
reference itself in the build container (tests/golden/make_golden.py, which imports
/root/reference with restated PyG 2.1.0 / torch_scatter 2.1.0 semantics; the reference has no
tests or fixtures of its own), see tests/test_oracle.py.

* ``triplets``  — vertex_to_edge_2 (edge_graph.py:12-30), numpy + a brute-force enumerator
* ``ref_cpu``   — xgnn_poly / xgnn_poly_global forward (xgnn.py, model.py, sbftransformer_conv.py,
                  readout.py, residual_layer.py, atom_embedding.py, envelop.py,
                  radial_basis_layer.py, angular_basis_layer.py) in torch-CPU fp32 with the
                  PyG/torch_scatter operators restated (index_select lift, index_add scatter,
                  segment-max softmax, graph-mode LayerNorm)
"""
