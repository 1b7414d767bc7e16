"""ctypes binding of libx2g.so (the C ABI declared in include/x2g.h).

The library is loaded after ``torch`` so that it binds to the HIP runtime PyTorch already
loaded (same soname), and every call is enqueued on PyTorch's current stream.  There is no
fallback: if the library or a GPU is missing, the product path raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must be imported before the HIP library is loaded)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("X2G_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libx2g.so"))

_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name -> argtypes (restype int unless noted); mirrors include/x2g.h
SIGNATURES = {
    "x2g_abi_version": [],
    "x2g_status_string": [ctypes.c_int],
    "x2g_csr_rowptr": [_P, _I64, _I64, _P, _P],
    "x2g_vertex_to_edge_workspace": [_I64, _I64],
    "x2g_vertex_to_edge": [_P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P],
    "x2g_line_graph_transpose": [_P, _P, _I64, _I64, _P, _P, _P, _P, _SZ, _P],
    "x2g_bessel_env": [_P, _I64, _F, _I32, _I32, _P, _P],
    "x2g_edge_basis": [_P, _P, _P, _I64, _F, _P, _I32, _I32, _I32, _P, _P, _P, _P, _P],
    "x2g_edge_basis_freq_grad_workspace": [_I64, _I32],
    "x2g_edge_basis_freq_grad_splits": [_I64],
    "x2g_edge_basis_freq_grad": [_P, _P, _P, _P, _I64, _I32, _F, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_keyed_row_sum_workspace": [_I64, _I32, _I32],
    "x2g_residual_fwd": [_P, _P, _P, _P, _P, _I64, _I32, _P, _P, _P, _P, _P],
    "x2g_dense_fwd_batched": [_P, _I32, _I64, _I32, _I32, ctypes.c_int, _P],
    "x2g_dense_bwd_batched": [_P, _I32, _I64, _I32, _I32, ctypes.c_int, ctypes.c_int, _P, _SZ, _P],
    "x2g_readout_head_fwd": [_P, _I32, _I64, _I32, _P, _P],
    "x2g_readout_head_pool_fwd": [_P, _I32, _I64, _I32, _P, _I64, _P, _P],
    "x2g_readout_head_pool_bwd": [_P, _P, _I64, _P, _I32, _I64, _I32, ctypes.c_int, _P, _SZ, _P],
    "x2g_readout_head_bwd_workspace": [_I64, _I32, _I32],
    "x2g_readout_head_bwd_splits": [_I64],
    "x2g_readout_head_bwd": [_P, _P, _I32, _I64, _I32, ctypes.c_int, _P, _SZ, _P],
    "x2g_embedding_table": [_P, _P, _I64, _I32, _I32, _F, _P, _P, _P],
    "x2g_embedding_table_bwd": [_P, _P, _I32, _I32, _I32, _P, ctypes.c_int, _P],
    "x2g_keyed_row_sum": [_P, _P, _I64, _I32, _I32, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_rbf_gate_fwd": [_P, _P, _P, _P, _I64, _I32, _I32, _P, _P],
    "x2g_rbf_pool_fwd": [_P, _P, _P, _P, _P, _I64, _I32, _I32, _P, _P],
    "x2g_rbf_gate_bwd_workspace": [_I64, _I32, _I32],
    "x2g_batch_meta": [_P, _P, _P, _I64, _I64, _I64] + [_P] * 9 + [_P],
    "x2g_vertex_to_edge_sym": [_P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _SZ, _P],
    "x2g_line_graph_transpose_sym": [_P, _P, _P, _P, _I64, _P, _P, _P, _P, _SZ, _P],
    "x2g_line_graph_sym_build": [_P, _P, _I64, _I64, _I64] + [_P] * 12 + [_P, _SZ, _P],
    "x2g_vertex_to_edge_sym_mol": [_P, _P, _I64, _I64, _I64, _P, _P, _P, _I64, _I32] + [_P] * 9 + [_P],
    "x2g_keyed_row_sum_batch_workspace": [_I64, _I32, _I32, _I32],
    "x2g_keyed_row_sum_batch": [_P, _P, _I32, _P, _I64, _I32, _I32, ctypes.c_int, _P, _SZ, _P],
    "x2g_clip_adam_ema_ex": [_P, _P, _P, _P, _P, _I64, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_rbf_pool_fwd_batch": [_P, _I32, _P, _P, _I64, _I32, _I32, _P],
    "x2g_rbf_gate_bwd_batch_workspace": [_I64, _I32, _I32, _I32],
    "x2g_rbf_gate_bwd_batch": [_P, _I32, _P, _P, _I64, _I32, _I32, _P, ctypes.c_int, _P, _P, _SZ, _P],
    "x2g_rbf_gate_bwd_splits": [_I64],
    "x2g_rbf_gate_bwd": [_P, _P, _P, _P, _P, _P, _I64, _I32, _I32, _P, _P, _P, _P, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_spherical_basis": [_P, _P, _P, _P, _P, _P, _P, _I64, _I32, _I32, _P, _P, _P, _P],
    "x2g_sbf_attention_bwd_dst_g": [_P, _P, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32,
                                    _I32, _P, _P, _P, _P, _P, _P],
    "x2g_sbf_attention_bwd_src_fold": [_P, _P, _P, _P, _P, _I32, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                       _P, _I64, _I64, _I32, _I32, _P, _P, _P, _P],
    "x2g_sbf_radial_wgrad_splits": [_I64],
    "x2g_sbf_radial_wgrad_workspace": [_I64, _I32],
    "x2g_sbf_radial_wgrad": [_P, _P, _I64, _I32, _P, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_sbf_attention_fwd": [_P, _P, _P, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _I64, _I64, _I32, _I32,
                              _I32, _P, _P, _P, _P, _P],
    "x2g_sbf_attention_fwd_stats": [_P, _P, _P, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _I64, _I64, _I32,
                                    _I32, _I32, _P, _P, _P, _P, _P, _P],
    "x2g_sbf_attention_fwd_center": [_P, _P, _P, _P, _P, _P, ctypes.c_int, _P, _I64, _P, _P, _P, _P, _I64, _I64, _I32,
                                     _I64, _I64, _I32, _I32, _P, _P, _P, _P, _P, _P],
    "x2g_sbf_attention_fwd_center_sf": [_P] * 6 + [ctypes.c_int] + [_P] * 10 + [_I64, _I64, _I32, _I64, _I64, _I32,
                                                                                _I32] + [_P] * 8,
    "x2g_sbf_attention_fwd_center_sf_tiled": [_P] * 6 + [ctypes.c_int] + [_P] * 10 + [_I64, _I64, _I32, _I32, _I64,
                                                                                      _I64, _I32, _I32] + [_P] * 8,
    "x2g_sbf_attention_fwd_center_sf_tiled_lds": [],
    "x2g_center_schedule_workspace": [_I64],
    "x2g_center_packs_host": [_P, _I64, _I32, _I32, _P, _P, _P, _P],
    "x2g_center_schedule": [_P, _P, _I64, _P, _P, _P, _P, _P, _SZ, _P],
    "x2g_sbf_attention_bwd_center_lds": [_I32, _I32],
    "x2g_sbf_attention_bwd_center": [_P] * 5 + [ctypes.c_int] + [_P] * 12 + [_I64, _I32, _I64, _I64, _I32, _I32] +
                                    [_P] * 7,
    "x2g_sbf_attention_bwd_dst": [_P, _P, _P, _P, _P, ctypes.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64,
                                  _I32, _I32, _I32, _P, _P, _P, _P, _P],
    "x2g_sbf_attention_bwd_src": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I64, _I64, _I32, _I32, _I32, _P,
                                  _P, _P],
    "x2g_segment_sum": [_P, _P, _P, _I64, _I64, _P, _P],
    "x2g_segment_broadcast": [_P, _P, _P, _I64, _I64, _P, _P],
    "x2g_segment_softmax_fwd": [_P, _P, _I64, _I64, _P, _P],
    "x2g_segment_softmax_bwd": [_P, _P, _P, _I64, _I64, _P, _P],
    "x2g_csr_rowptr_checked": [_P, _I64, _I64, _P, _P, _P],
    "x2g_segment_reduce_perm": [_P, _P, _P, _I64, _I64, ctypes.c_int, _P, _P],
    "x2g_segment_reduce_perm_bwd": [_P, _P, _P, _I64, _I64, ctypes.c_int, _P, _P],
    "x2g_segment_softmax_perm_fwd": [_P, _P, _P, _I64, _I64, _P, _P],
    "x2g_segment_softmax_perm_bwd": [_P, _P, _P, _P, _I64, _I64, _P, _P],
    "x2g_graph_layernorm_fwd": [_P, _P, _I64, _I64, _F, _P, _P, _P, _P],
    "x2g_graph_layernorm_bwd": [_P, _P, _P, _P, _I64, _I64, _P, _P],
    "x2g_graph_layernorm_bwd_workspace": [_I64],
    "x2g_chain_fwd_batch": [_P, _I32, _I32, _I64, _I32, _P],
    "x2g_smooth_l1_mean_fwd": [_P, _P, _I64, _F, _P, _P],
    "x2g_smooth_l1_mean_fwd_grad": [_P, _P, _I64, _F, _P, _P, _P],
    "x2g_smooth_l1_mean_bwd": [_P, _P, _I64, _F, _P, _P, _P],
    "x2g_chain_bwd_batch": [_P, _I32, _I32, _I64, _I32, _P],
    "x2g_graph_layernorm_bwd_ex": [_P, _P, _P, _P, _I64, _I64, _P, _P, _SZ, _P],
    "x2g_graph_layernorm_bwd_rows": [_P, _P, _P, _P, _I64, _I64, _P, _P, _P],
    "x2g_linear_wgrad_workspace": [_I64, _I32, _I32],
    "x2g_dense_fwd": [_P, _P, _P, _I64, _I32, _I32, ctypes.c_int, _P, _P, _P, _P],
    "x2g_dense_bwd_workspace": [_I64, _I32, _I32],
    "x2g_dense_bwd": [_P, _P, ctypes.c_int, _P, _P, _I64, _I32, _I32, _P, _P, _P, _P, _SZ, _P],
    "x2g_linear_wgrad_ex": [_P, _P, _I64, _I32, _I32, _P, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_optimizer_workspace": [_I64],
    "x2g_slab_sum_batch": [_P, _I32, _I32, _P],
    "x2g_linear_wgrad_splits": [_I64, _I32, _I32],
    "x2g_dense_bwd_splits": [_I64, _I32, _I32],
    "x2g_dense_bwd_slab_offset": [_I64, _I32, _I32],
    "x2g_sbf_project": [_P, _I64, _I32, _P, _P, _I32, _P, _P],
    "x2g_sbf_project_batch": [_P, _I64, _I32, _P, _P, _I32, _I32, _P, _P],
    "x2g_clip_adam_ema": [_P, _P, _P, _P, _P, _I64, _P, _P, _SZ, _P],
    "x2g_dense_bwd_ex": [_P, _P, ctypes.c_int, _P, _P, _I64, _I32, _I32, _P, _P, _P, _P, ctypes.c_int, _P, _SZ,
                         _P],
    "x2g_chain_fwd": [_P, _P, _P, _I32, _I64, _I32, _P, _P],
    "x2g_chain_fwd_ln": [_P, _P, _P, _I64, ctypes.c_float, _P, _P, _P, _P, _P, _I32, _I64, _I32, _P, _P],
    "x2g_chain_bwd": [_P, _P, _P, _I32, _I64, _I32, _P, _P, _P, _P],
    "x2g_chain_bwd_ln": [_P, _P, _P, _I32, _I64, _I32, _P, _P, _P, _P, _P, _P],
    "x2g_chain_t_floats": [_I64, _I32],
    "x2g_chain_wgrad_workspace": [_I64, _I32, _I32],
    "x2g_chain_wgrad": [_P, _P, _I32, _I64, _I32, _P, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_conv_proj_fwd": [_P, _P, _I32, _P, _P, _I64, _I32, _P, _P, _P],
    "x2g_conv_proj_bwd_gate_splits": [_I64],
    "x2g_conv_proj_bwd_gate_workspace": [_I64, _I32],
    "x2g_conv_proj_bwd_gate": [_P, _I64, _I32, _P, _P, _I32, _P, _P, _P, _P, _P, ctypes.c_int, _P, _SZ, _P],
    "x2g_tiled_wgrad_workspace": [_I64, _I32, _I32],
    "x2g_tiled_wgrad": [_P, _I32, _I64, _I32, ctypes.c_int, _P, _SZ, _P],
    "x2g_table_chain_fwd": [_P, _I64, _I32, _P, _I32, _P],
    "x2g_table_chain_bwd_workspace": [_I32],
    "x2g_table_chain_bwd_ex": [_P, _I32, _I64, _I32, _P, _P, _SZ, _P],
    "x2g_tiled_wgrad_flat_workspace": [_I64, _I32, _I32],
    "x2g_tiled_wgrad_flat_rows_workspace": [_P, _I32, _I32],
    "x2g_tiled_wgrad_flat": [_P, _I32, _I64, _I32, ctypes.c_int, _P, _P, _SZ, _P],
    "x2g_tiled_wgrad_flat_rows": [_P, _P, _I32, _I32, ctypes.c_int, _P, _P, _SZ, _P],
    "x2g_feat_fwd": [_P, _P, _I64, _I32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "x2g_feat_bwd": [_P, _P, _P, _P, _I64, _P, _P, _P],
    "x2g_wgrad_batched_workspace": [_I64, _I32, _I32],
    "x2g_wgrad_batched_splits": [_I64, _I32, _I32],
    "x2g_wgrad_batched": [_P, _I32, _I64, _I32, ctypes.c_int, _P, _SZ, _P],
}
RESTYPES = {"x2g_status_string": ctypes.c_char_p, "x2g_vertex_to_edge_workspace": _SZ,
            "x2g_table_chain_bwd_workspace": _SZ,
            "x2g_linear_wgrad_workspace": _SZ, "x2g_dense_bwd_workspace": _SZ, "x2g_optimizer_workspace": _SZ,
            "x2g_linear_wgrad_splits": ctypes.c_int32, "x2g_dense_bwd_splits": ctypes.c_int32,
            "x2g_dense_bwd_slab_offset": ctypes.c_int64, "x2g_edge_basis_freq_grad_workspace": _SZ,
            "x2g_edge_basis_freq_grad_splits": ctypes.c_int32, "x2g_rbf_gate_bwd_workspace": _SZ, "x2g_rbf_gate_bwd_batch_workspace": _SZ, "x2g_keyed_row_sum_batch_workspace": _SZ,
            "x2g_rbf_gate_bwd_splits": ctypes.c_int32, "x2g_keyed_row_sum_workspace": _SZ,
            "x2g_readout_head_bwd_workspace": _SZ, "x2g_readout_head_bwd_splits": ctypes.c_int32,
            "x2g_sbf_radial_wgrad_splits": ctypes.c_int32, "x2g_sbf_radial_wgrad_workspace": _SZ,
            "x2g_wgrad_batched_workspace": _SZ, "x2g_wgrad_batched_splits": ctypes.c_int32,
            "x2g_chain_t_floats": ctypes.c_int64, "x2g_chain_wgrad_workspace": _SZ,
            "x2g_tiled_wgrad_workspace": _SZ, "x2g_tiled_wgrad_flat_workspace": _SZ,
            "x2g_tiled_wgrad_flat_rows_workspace": _SZ,
            "x2g_conv_proj_bwd_gate_splits": ctypes.c_int32,
            "x2g_conv_proj_bwd_gate_workspace": _SZ, "x2g_graph_layernorm_bwd_workspace": _SZ,
            "x2g_sbf_attention_bwd_center_lds": _SZ, "x2g_sbf_attention_fwd_center_sf_tiled_lds": _SZ,
            "x2g_center_schedule_workspace": _SZ}

_lib = None


def load():
    """Load libx2g.so and declare every entry point (raises if the library is missing)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libx2g.so not found at {LIB_PATH}: build it (make -C x2-gnn_amd) first")
        lib = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = args
            fn.restype = RESTYPES.get(name, ctypes.c_int)
        _lib = lib
    return _lib


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def check(rc: int, name: str):
    if rc != 0:
        msg = load().x2g_status_string(rc).decode()
        raise RuntimeError(f"{name} failed with status {rc}: {msg}")


def call(name: str, *args):
    check(getattr(load(), name)(*args), name)
