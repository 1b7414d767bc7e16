/*
 * x2g.h — C ABI of libx2g.so, the MI355X (gfx950) kernels behind X2-GNN's message-passing
 * hot path.  Plain pointers and sizes only; no torch / HIP types in the signatures.
 *
 * Conventions:
 *  - every pointer is a DEVICE pointer that stays valid until the work enqueued on `stream`
 *    completes; `stream` is a hipStream_t passed as void* (NULL = default stream);
 *  - the library never allocates or frees: outputs and workspaces are caller-owned
 *    (the Python host layer allocates them from PyTorch's caching allocator);
 *  - index arrays are int32; float tensors are fp32, row-major, contiguous;
 *  - functions only enqueue work: no host synchronisation, no device->host reads; every size
 *    comes from the caller;
 *  - return 0 on success, a hipError_t value on a launch failure, or an X2G_E* code below;
 *    never abort, never throw across the ABI;
 *  - results are deterministic: segmented reductions run in a fixed order, no float atomics.
 *
 * Each entry point names the reference interface it replaces (file:line in zfwangDP/X2-GNN,
 * plus the un-vendored torch_scatter 2.1.0 / PyG 2.1.0 operators it reached).
 */
#ifndef X2G_H
#define X2G_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define X2G_OK 0
#define X2G_EINVAL 1001        /* bad size / null pointer */
#define X2G_EUNSUPPORTED 1002  /* shape outside the compiled kernel set */
#define X2G_EWORKSPACE 1003    /* workspace too small */

/* edge-term modes of the attention kernels */
#define X2G_EDGE_NONE 0        /* edge_dim=None: no lin_edge term */
#define X2G_EDGE_PER_TRIPLET 1 /* edge[T, H*C]: one row per triplet (reference layout) */
#define X2G_EDGE_PER_DST 2     /* edge[R, H*C] indexed by edge_row[E]: one row per destination line node */

int x2g_abi_version(void);
const char* x2g_status_string(int status);

/* ---------------------------------------------------------------- line graph (triplets) */

/* rowptr[s] = first i with keys[i] >= s, for s in [0, n_seg]; keys sorted ascending.
 * Replaces the CSR row pointer scipy builds in edge_graph.py:14 (adj_matrix.tocsr()). */
int x2g_csr_rowptr(const int32_t* keys, int64_t n, int64_t n_seg, int32_t* rowptr, void* stream);

/* The same row pointer for keys the caller only ASSUMES sorted (the drop-in APIs' sync-free
 * path, sbftransformer_conv.py:109 propagate over edge_index[1]; model.py:46,53 batch vectors):
 * rowptr[s] = lower_bound(keys, s) by binary search, so every entry is written and lies in
 * [0, n] whatever the keys hold, and status[0] is set to 1 (vector store, no host read) when a key
 * is out of [0, n_seg) or smaller than its predecessor; status[0] is zeroed first.  A violated
 * contract therefore gives wrong numbers, flagged on the device, never an out-of-range access. */
int x2g_csr_rowptr_checked(const int32_t* keys, int64_t n, int64_t n_seg, int32_t* rowptr, int32_t* status,
                           void* stream);

/* Workspace bytes for x2g_vertex_to_edge / x2g_line_graph_transpose. */
size_t x2g_vertex_to_edge_workspace(int64_t num_edges, int64_t num_nodes);

/* vertex_to_edge_2 (edge_graph.py:12-30): for every directed edge e=(a->b), in edge order, and
 * every k in N_out(b) ascending with k != a, emit triplet t with
 *   trip_src[t] = id(b->k), trip_dst[t] = e, atom_j[t] = b, atom_i[t] = a, atom_k[t] = k.
 * edge_src/edge_dst: int32[E], sorted by (src, dst) (np.argwhere order, atom_graph.py:42-45).
 * num_triplets must equal the true count (host metadata); trip_rowptr[E+1] receives the
 * CSR-by-destination row pointer; atom_rowptr[N+1] the source-atom CSR of the edges.
 * Any of atom_j/atom_i/atom_k may be NULL. */
int x2g_vertex_to_edge(const int32_t* edge_src, const int32_t* edge_dst, int64_t num_edges,
                       int64_t num_nodes, int64_t num_triplets, int32_t* atom_rowptr,
                       int32_t* trip_rowptr, int32_t* trip_src, int32_t* trip_dst, int32_t* atom_j,
                       int32_t* atom_i, int32_t* atom_k, void* workspace, size_t workspace_bytes,
                       void* stream);

/* Triplets regrouped by source line node (the transpose the backward of the k_j / v_j gathers
 * needs): src_rowptr[E+1]; src_perm[T] lists triplet ids of each source in ascending order;
 * src_dst[T] (optional, NULL = not written; needs trip_dst) = trip_dst[src_perm[p]], the destination of
 * each source-major position, so the source pass reaches it in one hop.
 * Replaces the atomics of ATen index_add_ behind PyG's index_select backward. */
int x2g_line_graph_transpose(const int32_t* trip_src, const int32_t* trip_dst, int64_t num_triplets,
                             int64_t num_edges, int32_t* src_rowptr, int32_t* src_perm, int32_t* src_dst,
                             void* workspace, size_t workspace_bytes, void* stream);

/* The same two operations for a SYMMETRIC edge set (b->a present for every a->b, as every
 * molecular graph: atom_graph.py:42-45 builds it from a symmetric distance test); the caller
 * asserts it (x2gnn's collate checks it on the host).  Per-edge counts are then degrees (deg(b) - 1
 * triplets per destination a->b and per source b->k), so count and scan are one launch, and the
 * transposed lists are written in order directly (no atomics, no segment sort).  Outputs equal
 * x2g_vertex_to_edge's / x2g_line_graph_transpose's bit for bit on such graphs. */
/* edge_rev / rev_trip (both or neither; NULL = not written), for the center-atom attention kernels:
 * edge_rev[e] = id(b->a) for e = (a->b) (the neighbour vertex_to_edge_2 excludes), and
 * rev_trip[id(b->a)] = trip_rowptr[e] — per source line node s, where the triplet block of its reverse
 * edge starts. */
int x2g_vertex_to_edge_sym(const int32_t* edge_src, const int32_t* edge_dst, int64_t num_edges, int64_t num_nodes,
                           int64_t num_triplets, int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src,
                           int32_t* trip_dst, int32_t* atom_j, int32_t* atom_i, int32_t* atom_k, int32_t* edge_rev,
                           int32_t* rev_trip, void* workspace, size_t workspace_bytes, void* stream);
int x2g_line_graph_transpose_sym(const int32_t* edge_src, const int32_t* edge_dst, const int32_t* atom_rowptr,
                                 const int32_t* trip_rowptr, int64_t num_edges, int32_t* src_rowptr,
                                 int32_t* src_perm, int32_t* src_dst, void* workspace, size_t workspace_bytes,
                                 void* stream);
/* x2g_vertex_to_edge_sym for a BATCH OF MOLECULES (every edge joins two atoms of one molecule, as in a
 * PyG batch): the atom and triplet row pointers one workgroup per molecule (its atoms mol_ptr[m] ..
 * mol_ptr[m+1]-1 own its edges line_ptr[m] .. line_ptr[m+1]-1; the triplets before it sum_{m'<m}
 * mol_trips[m'], int64 [num_mols]: the host's per-molecule counts or x2g_batch_meta's), then the same
 * emission: two launches, no scan over the whole batch, no workspace; outputs equal x2g_vertex_to_edge_sym's
 * bit for bit.  max_mol_atoms >= every molecule's atom count (<= 16384: it sizes a degree histogram in
 * LDS), T < 2^31, else X2G_EUNSUPPORTED.  The transpose, when a backward needs it, comes from
 * x2g_line_graph_transpose_sym. */
int x2g_vertex_to_edge_sym_mol(const int32_t* edge_src, const int32_t* edge_dst, int64_t num_edges,
                               int64_t num_nodes, int64_t num_triplets, const int32_t* mol_ptr,
                               const int32_t* line_ptr, const int64_t* mol_trips, int64_t num_mols,
                               int32_t max_mol_atoms, int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src,
                               int32_t* trip_dst, int32_t* atom_j, int32_t* atom_i, int32_t* atom_k,
                               int32_t* edge_rev, int32_t* rev_trip, void* stream);
/* Both at once for a training batch (a backward will need the transpose): x2g_vertex_to_edge_sym's
 * outputs and x2g_line_graph_transpose_sym's (src_rowptr [E+1], src_perm [T], src_dst [T] or NULL) in
 * three launches instead of five — the source row pointer from the same one-workgroup scan, the
 * emission and the transpose in one grid.  Outputs equal the two entry points' bit for bit. */
int x2g_line_graph_sym_build(const int32_t* edge_src, const int32_t* edge_dst, int64_t num_edges, int64_t num_nodes,
                             int64_t num_triplets, int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src,
                             int32_t* trip_dst, int32_t* atom_j, int32_t* atom_i, int32_t* atom_k,
                             int32_t* src_rowptr, int32_t* src_perm, int32_t* src_dst, int32_t* edge_rev,
                             int32_t* rev_trip, void* workspace, size_t workspace_bytes, void* stream);

/* Size metadata and int32 index forms of a PyG-style batch from its tensors, on the device (for a Batch
 * made elsewhere, e.g. by the reference trainer's DataLoader, trainer.py:25-27,37-40, which carries no
 * triplet counts; xgnn.py:41-52), in one pass and no host loop: from edge_index (int64 [2, E], PyG), x
 * (int64 [N], atomic numbers) and batch (int64 [N], the molecule of each atom; NULL = one molecule):
 * edge_src / edge_dst (int32 [E]), their elements src_type / dst_type (int32 [E]), atom_type (int32 [N]),
 * the molecules' atom and edge row pointers mol_ptr / line_ptr (int32 [num_graphs + 1]), atom_rowptr
 * [N+1] of edge_src, and everything the host needs in one int64 block (one copy back):
 * info = [mol_ptr (B+1) | line_ptr (B+1) | triplets (B) | flags (4)], B = num_graphs, where triplets[g] =
 * sum over molecule g's edges e = (a->b) of |N_out(b) \ {a}| and flags = [edges whose reverse is missing
 * (0 = a symmetric edge set), the largest out-degree, edges out of (src, dst) order / repeated / out of
 * range, edges joining two molecules (0 = x2g_vertex_to_edge_sym_mol applies)].  Integer atomics only:
 * exact. */
int x2g_batch_meta(const int64_t* edge_index, const int64_t* x, const int64_t* batch, int64_t num_edges,
                   int64_t num_nodes, int64_t num_graphs, int32_t* edge_src, int32_t* edge_dst, int32_t* src_type,
                   int32_t* dst_type, int32_t* atom_type, int32_t* line_ptr, int32_t* mol_ptr, int32_t* atom_rowptr,
                   int64_t* info, void* stream);

/* ---------------------------------------------------------------- basis (featurisation) */

/* rbf_env[e, l*R+n] = env(d_e) * N_ln j_l(z_ln d_e/cutoff)   (l < num_spherical, n < R = num_radial)
 * = the E-row part of F_B_2D(num_spherical, num_radial).forward (angular_basis_layer.py:51-86) with
 * poly_envelop (envelop.py:16-21, exponent 5).  Compiled for num_spherical <= 7, num_radial <= 16
 * (config.json: 7 x 6; the reference's default xgnn_poly: 7 x 16, xgnn.py:16), else X2G_EUNSUPPORTED. */
int x2g_bessel_env(const float* dist, int64_t num_edges, float cutoff, int32_t num_spherical, int32_t num_radial,
                   float* rbf_env, void* stream);

/* The whole E-row featurisation in one launch (xgnn.py:49-53 + radial_basis_layer.py:36-40 +
 * envelop.py:16-21 + the E-row half of angular_basis_layer.py:80-86), per directed edge e = (a, b):
 *   dist[e] = |pos[a] - pos[b]|,  env[e] = poly_envelop(dist / cutoff) (exponent 5),
 *   rbf_env[e, n] = sin(freq[n] * dist / cutoff) * env[e]   (n < num_freq <= 16; the trainable
 *                   RadialBasis times the envelope: xgnn_poly's node_rbf),
 *   bessel_env[e, :] = x2g_bessel_env's num_spherical * num_radial values (optional, NULL skips).
 * edge_src/edge_dst int32 atom ids. */
int x2g_edge_basis(const float* pos, const int32_t* edge_src, const int32_t* edge_dst, int64_t num_edges,
                   float cutoff, const float* freq, int32_t num_freq, int32_t num_spherical, int32_t num_radial,
                   float* dist, float* env, float* rbf_env, float* bessel_env, void* stream);

/* d loss / d freq[n] = sum_e g[e, n] * env[e] * cos(freq[n] x_e) * x_e, x_e = dist[e] / cutoff
 * (the backward of rbf_env w.r.t. RadialBasis.frequencies).  Deterministic: per-workgroup
 * partials + a fixed-order sum; flags X2G_ACCUM_WGRAD (dfreq +=) and X2G_DEFER_SLAB_SUM (leave
 * the partials for x2g_slab_sum_batch: x2g_edge_basis_freq_grad_splits slabs of num_radial floats
 * at the start of the workspace). */
size_t x2g_edge_basis_freq_grad_workspace(int64_t num_edges, int32_t num_radial);
int32_t x2g_edge_basis_freq_grad_splits(int64_t num_edges);
int x2g_edge_basis_freq_grad(const float* g, const float* dist, const float* env, const float* freq,
                             int64_t num_edges, int32_t num_radial, float cutoff, float* dfreq, int flags,
                             void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- element embedding table
 * EmbeddingBlock's Embedding(num_embeddings, D, padding_idx, max_norm, scale_grad_by_freq)
 * (atom_embedding.py:13-25) evaluated once per ELEMENT instead of per atom:
 *   counts[v] = #{n : z[n] == v}  (exact, integer atomics),
 *   rows v with counts[v] > 0 and ||weight[v]||_2 > max_norm are rescaled IN PLACE by
 *   max_norm / (norm + 1e-7)  (torch.embedding_renorm_; max_norm <= 0 disables),
 *   table[v, :] = weight[v, :] after the renorm.
 * z: int64 atomic numbers in [0, V), V <= 64.  One workgroup. */
int x2g_embedding_table(float* weight, const int64_t* z, int64_t num_atoms, int32_t num_embeddings, int32_t dim,
                        float max_norm, float* counts, float* table, void* stream);

/* d weight[v, :] (+)= g[v, :] / max(counts[v], 1)  (scale_grad_by_freq; counts NULL: no scaling),
 * zero for v == padding_idx (< 0: none); flags X2G_ACCUM_WGRAD (+=). */
int x2g_embedding_table_bwd(const float* g, const float* counts, int32_t num_embeddings, int32_t dim,
                            int32_t padding_idx, float* dweight, int flags, void* stream);

/* ---------------------------------------------------------------- rbf gates (x * lin_rbf(rbf))
 * f[e, c] = sum_j w[c, j] rbf[e, j] + b[c]   (w [D, R] row-major, R <= 8, b optional; D % 4 == 0)
 * gate:  out[e, :] = x[e, :] * f[e, :]                 (SBFTransformerConv x_src,
 *                                                       sbftransformer_conv.py:99-101)
 * pool:  out[n, :] = sum_{e in [rowptr[n], rowptr[n+1])} x[e, :] * f[e, :]
 *        (AtomWise / MolWise edge->atom pooling, readout.py:39-41,66-67; rows sorted by owner)
 * The [E, D] filter f is never materialised. */
int x2g_rbf_gate_fwd(const float* x, const float* rbf, const float* w, const float* b, int64_t rows, int32_t D,
                     int32_t R, float* out, void* stream);
int x2g_rbf_pool_fwd(const float* x, const float* rbf, const float* w, const float* b, const int32_t* rowptr,
                     int64_t num_segments, int32_t D, int32_t R, float* out, void* stream);

/* Backward of both: g_row(e) = g[e] (gate, owner == NULL) or g[owner[e]] (pool):
 *   dx[e] = g_row * f[e] (+ dx_add[e]; dx may alias dx_add),  drbf[e, j] (+)= sum_c (g_row x[e])_c w[c, j]
 *   (added to drbf's contents with flags X2G_GATE_DRBF_ACCUM: the rbf feeds every layer's gate),
 *   dw[c, j] (+)= sum_e (g_row x[e])_c rbf[e, j],  db[c] (+)= sum_e (g_row x[e])_c   (db optional).
 * dx / drbf may be NULL (not needed).  Weight gradients: per-workgroup partials + fixed-order
 * sum, flags as x2g_linear_wgrad_ex (slabs of D*R then D floats at the start of the workspace). */
#define X2G_GATE_DRBF_ACCUM 4
size_t x2g_rbf_gate_bwd_workspace(int64_t rows, int32_t D, int32_t R);
int32_t x2g_rbf_gate_bwd_splits(int64_t rows);
int x2g_rbf_gate_bwd(const float* g, const int32_t* owner, const float* x, const float* rbf, const float* w,
                     const float* b, int64_t rows, int32_t D, int32_t R, float* dx, const float* dx_add,
                     float* drbf, float* dw, float* db, int flags, void* workspace, size_t workspace_bytes,
                     void* stream);

/* sbf[t, l*R+n] = rbf_env[trip_src[t], l*R+n] * Y_l0(theta_t)  (R = num_radial; shapes as x2g_bessel_env), theta_t = atan2(|ji x jk|, ji.jk),
 * ji = pos[atom_i]-pos[atom_j], jk = pos[atom_k]-pos[atom_j]  (xgnn.py:61-65,
 * angular_basis_layer.py:87-93).  If theta[T] is non-NULL it is used instead of the positions
 * (F_B_2D.forward(d, Angles, edge_index_1) signature; pos/atom_* may then be NULL).
 * cos_theta[T] (optional, may be NULL) receives cos(theta).  sph_y[T, 8] (optional, 16-byte
 * aligned) receives Y_0..Y_6 (theta_t) and a 1: the angular factor of sbf, which the factorised
 * lin_sbf backward (x2g_sbf_attention_bwd_src_fold) folds per triplet.  sbf may be NULL when sph_y is
 * given (the factors alone: the center-atom forward rebuilds lin_sbf(sbf) from them). */
int x2g_spherical_basis(const float* pos, const int32_t* atom_i, const int32_t* atom_j,
                        const int32_t* atom_k, const float* theta, const int32_t* trip_src,
                        const float* rbf_env, int64_t num_triplets, int32_t num_spherical, int32_t num_radial,
                        float* sbf, float* cos_theta, float* sph_y, void* stream);

/* ---------------------------------------------------------------- SBF-transformer attention */

/* S[t, :] = w_sbf[out_dim, sbf_dim] sbf[t, :] + b_sbf: lin_sbf of sbftransformer_conv.py:148,
 * materialised once per layer so the attention kernels read one row per triplet instead of
 * re-projecting it.  sbf_dim 42 (config.json's 7 x 6 basis): out_dim in {32, 64, 128, 256} on the
 * compiled narrow-K kernels; any other sbf_dim (e.g. 112, the reference's default 7 x 16) runs as
 * x2g_dense_fwd. */
int x2g_sbf_project(const float* sbf, int64_t num_triplets, int32_t sbf_dim, const float* w_sbf,
                    const float* b_sbf, int32_t out_dim, float* sbfproj, void* stream);

/* Every layer's S_l = sbf W_l^T + b_l in one launch (layers 1..X2G_SBF_PROJECT_MAX_LAYERS; the
 * trunk's lin_sbf of every SBFTransformerConv, sbftransformer_conv.py:142): w_sbf / b_sbf / sbfproj are
 * HOST arrays of n_layers device pointers.  Each S_l equals x2g_sbf_project's bit for bit. */
#define X2G_SBF_PROJECT_MAX_LAYERS 8
int x2g_sbf_project_batch(const float* sbf, int64_t num_triplets, int32_t sbf_dim, const float* const* w_sbf,
                          const float* const* b_sbf, int32_t n_layers, int32_t out_dim, float* const* sbfproj,
                          void* stream);

/* In the three attention entry points below, w_sbf == NULL (and b_sbf == NULL) means `sbf` is
 * that precomputed projection S [T, heads*channels] and sbf_dim must equal heads*channels;
 * otherwise `sbf` is the raw basis [T, 42] and the projection is computed per triplet. */

/* Fused SBFTransformerConv.message + PyG softmax + 'add' aggregation + root skip
 * (sbftransformer_conv.py:109-127,138-162), CSR by destination:
 *   kk_t = k[src]+edge_t, u_t = v[src]+edge_t, alpha_t,h = <q[dst]_h, kk_t,h>/sqrt(C),
 *   a = softmax_dst(alpha) (max shift, /(sum+1e-16)), S_t = W_sbf sbf_t + b_sbf,
 *   out[e] = sum_{t in seg(e)} u_t*S_t*a_t,h + skip[e].
 * Saves alpha_raw[T,H], seg_max[E,H], seg_den[E,H] for the backward.
 * Compiled for H*C in {32,64,128,256}, C in {4,8,16,32} with C >= channels-per-lane, sbf_dim 42. */
int x2g_sbf_attention_fwd(const float* q, const float* k, const float* v, const float* skip,
                          const float* edge, const int32_t* edge_row, int edge_mode, const float* sbf,
                          const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                          const int32_t* trip_src, int64_t num_edges, int64_t num_triplets,
                          int32_t heads, int32_t channels, int32_t sbf_dim, float* out,
                          float* alpha_raw, float* seg_max, float* seg_den, void* stream);

/* The same forward, also writing row_stats[E, 2] = (mean of out[e, :], sum over c of (out[e, c] -
 * that mean)^2) per output row: the graph LayerNorm that follows the conv (model.py:46, PyG
 * LayerNorm(mode='graph')) is then fused into the next kernel's staging (x2g_chain_fwd_ln).
 * row_stats 8-byte aligned. */
int x2g_sbf_attention_fwd_stats(const float* q, const float* k, const float* v, const float* skip,
                                const float* edge, const int32_t* edge_row, int edge_mode, const float* sbf,
                                const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                                const int32_t* trip_src, int64_t num_edges, int64_t num_triplets,
                                int32_t heads, int32_t channels, int32_t sbf_dim, float* out,
                                float* alpha_raw, float* seg_max, float* seg_den, float* row_stats, void* stream);

/* The forward over a SYMMETRIC line graph grouped by center atom (csrc/attention_center.hip): the
 * triplets through atom b are the block {(b->k_j) -> (k_i->b) : i != j} over b's n = deg(b) neighbours,
 * so one workgroup per atom stages the n source rows of k and v (b's out-edges: contiguous line nodes)
 * in LDS once, coalesced, and destination i = edge_rev[b->k_i] streams its contiguous triplet rows
 * rev_trip[b->k_i] + 0 .. n-2.  Same outputs as x2g_sbf_attention_fwd(_stats) (row_stats may be NULL)
 * on such graphs, up to fp32 rounding (per-batch softmax rescale, 4-channel head sums).
 *   edge_mode X2G_EDGE_NONE or X2G_EDGE_PER_DST; for the latter the edge term of center atom b is row
 *   src_row[atom_rowptr[b]] of `edge` (X2-GNN: the element-table row of b, the per-source src_type).
 *   sbfproj: S rows for triplets t_base .. (row t - t_base), covering every triplet of the atoms
 *   atom0 .. atom0 + n_atoms - 1 (whole molecules: the tiled inference path passes a molecule range).
 *   max_degree >= every deg(b) of those atoms, <= X2G_CENTER_MAX_DEGREE (sizes the LDS image).
 *   atom_order (or NULL): workgroup w takes center atom atom_order[atom0 + w] (a permutation of the range;
 *   x2gnn passes the atoms by decreasing degree, so the longest blocks start first).
 *   alpha_raw may be NULL (inference without attention weights): the logits are then not stored.
 * heads * channels = 128 and channels a multiple of 4, 16-byte aligned rows, else X2G_EUNSUPPORTED. */
#define X2G_CENTER_MAX_DEGREE 128
int x2g_sbf_attention_fwd_center(const float* q, const float* k, const float* v, const float* skip,
                                 const float* edge, const int32_t* src_row, int edge_mode, const float* sbfproj,
                                 int64_t t_base, const int32_t* atom_rowptr, const int32_t* edge_rev,
                                 const int32_t* rev_trip, const int32_t* atom_order, int64_t atom0, int64_t n_atoms,
                                 int32_t max_degree,
                                 int64_t num_edges, int64_t num_triplets, int32_t heads, int32_t channels, float* out,
                                 float* alpha_raw, float* seg_max, float* seg_den, float* row_stats, void* stream);

/* The center-atom kernels' schedule made on the device, for a batch that does not carry collate's
 * (data.center_packs; the reference trainer's PyG batch, trainer.py:25-27,37-40): from the atoms' out-edge
 * row pointer atom_rowptr [N + 1] and src_row [E] (or NULL), writes
 *   center_order [N]: every atom by decreasing degree (the center backward's workgroups);
 *   pack_order [N], pack_ptr [N + 1], atom_info [N, 4] (16-byte aligned): the fused forward's units — per
 *   window of 64 consecutive atoms its atoms by decreasing degree packed best-fit into units of <= 16 rows and
 *   <= 16 atoms (an atom of degree >= 16 alone) — in one list by decreasing largest degree, units 0 .. U - 1,
 *   the slots U .. N - 1 empty (pack_ptr[s] == pack_ptr[s + 1] == N): launch the fused forwards over all N
 *   units (x2g_sbf_attention_fwd_center_sf with max_rows 17 leaves out the units of more rows,
 *   x2g_sbf_attention_fwd_center_sf_tiled with skip_rows 17 takes exactly those; the empty slots leave at once).
 * workspace: x2g_center_schedule_workspace(N) bytes, 8-byte aligned.  Three launches and a memset on the
 * stream, no host read.  The order among atoms (units) of equal degree follows integer atomics; no output of
 * the center kernels depends on it.  (ABI 17; ABI 16 took mol_ptr / num_graphs and left the units in
 * per-molecule slots.) */
/* HOST function (no device work, no stream): collate's center-kernel units (x2gnn.data.center_packs) for
 * the atom degrees deg [n]: the atoms by decreasing degree (ties by index) packed best-fit into units of
 * <= cap rows and <= max_members atoms (the fullest open unit that takes an atom, the most recently opened of
 * equally full ones; an atom of degree >= cap alone), atoms without edges max_members to a unit in index
 * order after all others; the units in the order they were opened.  Writes order [n], packs [units + 1]
 * (caller-sized n + 1), the unit count and the largest unit's row count. */
int x2g_center_packs_host(const int64_t* deg, int64_t n, int32_t cap, int32_t max_members, int32_t* order,
                          int32_t* packs, int64_t* n_units, int32_t* max_rows);
size_t x2g_center_schedule_workspace(int64_t num_atoms);
int x2g_center_schedule(const int32_t* atom_rowptr, const int32_t* src_row, int64_t num_atoms,
                        int32_t* center_order, int32_t* pack_order, int32_t* pack_ptr, int32_t* atom_info,
                        void* workspace, size_t ws_bytes, void* stream);

/* Workgroup UNITS of the fused-projection center forward below: with pack_ptr (int32 [units + 1], or NULL)
 * unit u is the PACK of center atoms atom_order[pack_ptr[u]] .. atom_order[pack_ptr[u + 1] - 1] (at most
 * 32 atoms; every atom of the batch in exactly one pack, atoms without edges included), processed side by
 * side by one workgroup (its 16 half-wave owners take the rows of all of them: x2gnn packs the atoms
 * best-fit-decreasing by degree into units of <= 16 rows, data.center_packs); without it unit u is atom
 * atom_order[u] (or u when atom_order is NULL).  max_rows >= the row count sum(deg) of every unit (the
 * largest degree without packs), <= X2G_CENTER_MAX_DEGREE: it sizes the LDS image.  Packing changes no
 * bit of any output (every sum keeps its order within an atom's block).  atom_info (or NULL): int32
 * [N, 4], 16-byte aligned, per position p of atom_order: (atom_order[p], atom_rowptr of it, its degree,
 * src_row of its first out-edge) — the workgroup then reads its atoms' row ranges with one load instead
 * of three dependent ones (x2gnn makes it at collate time).
 *
 * The center-atom forward with lin_sbf fused (no S to read): X2-GNN's sbf row factorises as
 * sbf[t, 6l+n] = R[s, 6l+n] Y_l(t) (angular_basis_layer.py:87-91; R = rbf_env [E, 42] of the triplet's
 * source s, Y = sph_y [T, 8] from x2g_spherical_basis), so S_t = b + sum_l Y_l(t) P_s[l] with
 * P_s[l][c] = sum_n W[c, 6l+n] R[s, 6l+n], formed per source in LDS for each center atom's block
 * (w_sbf [128, 42], b_sbf [128]).  Outputs as x2g_sbf_attention_fwd_center; for a backward, either
 * sbfproj_out [T, 128] receives every S_t row, or sbf_p_out [E, 7, 128] every source's P rows (3.5 KB per
 * line node instead of 512 B per triplet: x2g_sbf_attention_bwd_center rebuilds S_t from them bit for
 * bit); either may be NULL, and so may alpha_raw (inference: no logits stored).  Units unit0 .. unit0 +
 * n_units - 1.  LDS
 * per workgroup 4.7 KB x max_rows (<= 160 KiB, else X2G_EUNSUPPORTED); no t_base tiling is needed
 * (nothing T x 128 is read). */
int x2g_sbf_attention_fwd_center_sf(const float* q, const float* k, const float* v, const float* skip,
                                    const float* edge, const int32_t* src_row, int edge_mode, const float* radial,
                                    const float* sph_y, const float* w_sbf, const float* b_sbf,
                                    const int32_t* atom_rowptr, const int32_t* edge_rev, const int32_t* rev_trip,
                                    const int32_t* atom_order, const int32_t* pack_ptr, const int32_t* atom_info,
                                    int64_t unit0, int64_t n_units, int32_t max_rows, int64_t num_edges, int64_t num_triplets,
                                    int32_t heads, int32_t channels, float* out, float* alpha_raw, float* seg_max,
                                    float* seg_den, float* row_stats, float* sbfproj_out, float* sbf_p_out,
                                    void* stream);

/* The fused-projection center forward for atoms whose block exceeds that LDS image (config 5's AID atoms:
 * degrees up to 61; replaces the S = lin_sbf(sbf) projection + S-reading forward those took; reference
 * sbftransformer_conv.py:138-162, angular_basis_layer.py:86-93): one workgroup per unit, each unit a SINGLE
 * atom (atom_order[pack_ptr[u]], or atom_order[u] / u as above; atom_info as above), its sources staged 16 at
 * a time (k + e, v + e, radial rows, P rows in LDS: x2g_sbf_attention_fwd_center_sf_tiled_lds() bytes), the
 * 16 owners' destination rows d = owner + 16 r carrying their online-softmax state across the tiles; sources
 * in the same order, batches of 4 (equal to the untiled form to fp32 rounding).  max_degree >= every unit's
 * degree, <= X2G_CENTER_MAX_DEGREE.  skip_rows >= 0: units whose (first) atom has at most that many rows are
 * left to the untiled form (a list made by x2g_center_schedule mixes both kinds; x2gnn passes 17, the untiled
 * form's max_rows, which in turn leaves out every unit of more rows than its max_rows).  Outputs,
 * sbfproj_out / sbf_p_out and alpha_raw as the untiled form. */
size_t x2g_sbf_attention_fwd_center_sf_tiled_lds(void);
int x2g_sbf_attention_fwd_center_sf_tiled(const float* q, const float* k, const float* v, const float* skip,
                                          const float* edge, const int32_t* src_row, int edge_mode,
                                          const float* radial, const float* sph_y, const float* w_sbf,
                                          const float* b_sbf, const int32_t* atom_rowptr, const int32_t* edge_rev,
                                          const int32_t* rev_trip, const int32_t* atom_order,
                                          const int32_t* pack_ptr, const int32_t* atom_info, int64_t unit0,
                                          int64_t n_units, int32_t max_degree, int32_t skip_rows, int64_t num_edges,
                                          int64_t num_triplets, int32_t heads, int32_t channels, float* out,
                                          float* alpha_raw, float* seg_max, float* seg_den, float* row_stats,
                                          float* sbfproj_out, float* sbf_p_out, void* stream);

/* The whole attention backward over a SYMMETRIC line graph in ONE launch, one workgroup per center atom
 * (csrc/attention_center.hip): the block's rows (k + e of its sources, dout and q of its destinations,
 * their softmax max / denominator) staged in LDS, then per source j a pass over its triplets' S rows,
 * alpha (dv, and (g_t, a_t) pairs into the g_work scratch of 2 T heads floats), rho per destination, and per source /
 * destination dk, the folded lin_sbf gradient G (from Y) and dq.  Replaces x2g_sbf_attention_bwd_dst_g + x2g_sbf_attention_bwd_src_fold on such
 * graphs (same dq, dk, dv, radial_grad = G [E, 8, HC]; fp32 rounding apart), reading S once instead of
 * twice and no row gathers; d_edge_atom [num_atoms, HC] (or NULL) = the per-CENTER-ATOM gradient of the
 * edge term (sum over the atom's sources of dk + dv): the element-table gradient is its keyed sum by
 * atom element.  atom_order (or NULL): workgroup w takes atom atom_order[w] (x2gnn: by decreasing degree).
 * S_t comes from sbfproj [T, 128] rows, or (sbfproj NULL) from the fused forward's sbf_p [E, 7, 128] and
 * b_sbf [128] as S_t = b + sum_l Y_l(t) P_s[l] (exactly one of the two forms).  With sbf_p, alpha_raw is not
 * read (may be NULL): each logit is recomputed as q_i . (k_j + e) / sqrt(channels) in the forward's own
 * arithmetic, bit for bit, from rows the workgroup stages anyway.
 * sph_y [T, 8] as x2g_spherical_basis writes it.  LDS per workgroup:
 * x2g_sbf_attention_bwd_center_lds(max_degree, heads) bytes (<= 160 KiB, else X2G_EUNSUPPORTED).
 * heads * channels = 128, channels a multiple of 4, 16-byte aligned rows.  T-row arrays are addressed with
 * 32-bit offsets: T * 512 < 2^31 with sbfproj, T * heads * 8 < 2^31 with sbf_p, else X2G_EUNSUPPORTED
 * (x2gnn then takes the destination-major passes). */
size_t x2g_sbf_attention_bwd_center_lds(int32_t max_degree, int32_t heads);
int x2g_sbf_attention_bwd_center(const float* q, const float* k, const float* v, const float* edge,
                                 const int32_t* src_row, int edge_mode, const float* sbfproj, const float* sbf_p,
                                 const float* b_sbf, const float* sph_y,
                                 const int32_t* atom_rowptr, const int32_t* edge_rev, const int32_t* rev_trip,
                                 const int32_t* atom_order, const float* alpha_raw, const float* seg_max,
                                 const float* seg_den, const float* dout,
                                 int64_t num_atoms, int32_t max_degree, int64_t num_edges, int64_t num_triplets,
                                 int32_t heads, int32_t channels, float* dq, float* dk, float* dv, float* radial_grad,
                                 float* d_edge_atom, float* g_work, void* stream);
/* Backward, destination-major: dq[E,HC]; d_edge ([E,HC] per destination for EDGE_PER_DST,
 * [T,HC] for EDGE_PER_TRIPLET); dlogit[T,H] (grad of alpha_raw); d_sbfproj[T,HC] (grad of S_t,
 * so dW_sbf = d_sbfproj^T sbf and db_sbf = column sums). */
int x2g_sbf_attention_bwd_dst(const float* q, const float* k, const float* v, const float* edge,
                              const int32_t* edge_row, int edge_mode, const float* sbf,
                              const float* w_sbf, const float* b_sbf, const int32_t* trip_rowptr,
                              const int32_t* trip_src, const float* alpha_raw, const float* seg_max,
                              const float* seg_den, const float* dout, int64_t num_edges,
                              int64_t num_triplets, int32_t heads, int32_t channels, int32_t sbf_dim,
                              float* dq, float* d_edge, float* dlogit, float* d_sbfproj, void* stream);

/* Backward, source-major over x2g_line_graph_transpose's lists: dk[E,HC], dv[E,HC]
 * (the adjoint of PyG's index_select(key/value, edge_index[0]) lift, without atomics). */
int x2g_sbf_attention_bwd_src(const float* q, const float* sbf, const float* w_sbf,
                              const float* b_sbf, const int32_t* src_rowptr, const int32_t* src_perm,
                              const int32_t* trip_dst, const float* alpha_raw, const float* seg_max,
                              const float* seg_den, const float* dlogit, const float* dout,
                              int64_t num_edges, int64_t num_triplets, int32_t heads, int32_t channels,
                              int32_t sbf_dim, float* dk, float* dv, void* stream);

/* Factorised backward for X2-GNN's sbf = rbf_env[trip_src] * Y_l0(theta) (angular_basis_layer.py:87-91),
 * three launches instead of the two attention passes + the [T, HC] d_sbfproj + its T-row weight GEMM:
 *  (1) x2g_sbf_attention_bwd_dst_g: ONE pass per destination -> dq, d_edge (EDGE_NONE / EDGE_PER_DST
 *      only), g[T,H] = sum over the head's channels of dout (v[src]+edge) S_t (the softmax-output
 *      gradient), prob[T,H] = a_t (the softmax probabilities) and seg_rho[E,H] = sum_t a_t g_t;
 *      g_out may be NULL (not written: the source pass then recomputes g, bitwise the same value);
 *  (2) x2g_sbf_attention_bwd_src_fold: source-major -> dk, dv (dlogit = a (g - rho) formed here; g_in
 *      NULL: g recomputed from the rows the pass reads anyway, no [T, H] round trip) and
 *      radial_grad[E, 8, HC]: G[s, l, :] = sum_{t: src(t)=s} d_sbfproj[t, :] Y_l(t) (sph_y from
 *      x2g_spherical_basis; slot 7 = sum of d_sbfproj).  EDGE_PER_DST requires edge_row and a table
 *      of edge_rows <= 16 rows (staged in LDS), else X2G_EUNSUPPORTED;
 *  (3) x2g_sbf_radial_wgrad: dW_sbf[c, 6l+n] (+)= sum_s radial[s, 6l+n] G[s, l, c], db_sbf[c] (+)= sum_s
 *      G[s, 7, c]; radial = rbf_env [E, 42]; per-workgroup slabs + fixed-order sum, flags as
 *      x2g_linear_wgrad_ex (weight slabs then bias slabs at the start of the workspace).
 * sbfproj is the precomputed S = lin_sbf(sbf) [T, HC] (x2g_sbf_project). */
int x2g_sbf_attention_bwd_dst_g(const float* q, const float* k, const float* v, const float* edge,
                                const int32_t* edge_row, int edge_mode, const float* sbfproj,
                                const int32_t* trip_rowptr, const int32_t* trip_src, const float* alpha_raw,
                                const float* seg_max, const float* seg_den, const float* dout, int64_t num_edges,
                                int64_t num_triplets, int32_t heads, int32_t channels, float* dq, float* d_edge,
                                float* g_out, float* prob_out, float* seg_rho, void* stream);
/* Source pass options: src_dst[T] (x2g_line_graph_transpose*'s, may be NULL: then trip_dst[src_perm[p]]
 * is read, one more dependent hop); src_row[E] (EDGE_PER_DST only, may be NULL) = the edge row of
 * every triplet with source s, when it depends on s alone — true of the line graph x2g_vertex_to_edge
 * builds with the per-element table of xgnn.py:57-58 (the triplets of s = (b->k) share middle atom
 * b: src_row[s] = Z[b]); NULL = edge_row[trip_dst[t]] per triplet. */
int x2g_sbf_attention_bwd_src_fold(const float* q, const float* v, const float* edge, const int32_t* edge_row,
                                   const int32_t* src_row, int32_t edge_rows, int edge_mode, const float* sbfproj,
                                   const float* sph_y, const int32_t* src_rowptr, const int32_t* src_perm,
                                   const int32_t* src_dst, const int32_t* trip_dst, const float* prob,
                                   const float* g_in, const float* seg_rho, const float* dout, int64_t num_edges,
                                   int64_t num_triplets, int32_t heads, int32_t channels, float* dk, float* dv,
                                   float* radial_grad, void* stream);
int32_t x2g_sbf_radial_wgrad_splits(int64_t num_edges);
size_t x2g_sbf_radial_wgrad_workspace(int64_t num_edges, int32_t out_dim);
int x2g_sbf_radial_wgrad(const float* radial_grad, const float* radial, int64_t num_edges, int32_t out_dim,
                         float* dw, float* db, int flags, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- segmented reductions */

/* out[g, :] = sum_{r in [rowptr[g], rowptr[g+1])} x[r, :] (* mul[r, :] if mul != NULL).
 * torch_scatter scatter_add(src, index, dim=0, dim_size) for a sorted index
 * (readout.py:37, model.py:190, and the 'add' aggregation of MessagePassing). */
int x2g_segment_sum(const float* x, const float* mul, const int32_t* rowptr, int64_t num_segments,
                    int64_t dim, float* out, void* stream);

/* out[r, :] = g[seg(r), :] (* mul[r, :] if mul != NULL): adjoint of x2g_segment_sum. */
int x2g_segment_broadcast(const float* g, const float* mul, const int32_t* rowptr, int64_t num_segments,
                          int64_t dim, float* out, void* stream);

/* out[k, :] (+)= sum_{r : key[r] == k} src[r, :]  for an UNSORTED key in [0, num_keys), num_keys <= 16,
 * dim % 4 == 0, dim <= 256: the gradient of a row gather table[key] (the per-element edge table
 * that every triplet of destination e reads, xgnn.py:57-58 -> lin_edge, sbftransformer_conv.py:144).
 * Deterministic: per-workgroup partials in LDS (one accumulator set per row slot) + a fixed-order
 * sum; flags X2G_ACCUM_WGRAD (out +=). */
size_t x2g_keyed_row_sum_workspace(int64_t rows, int32_t dim, int32_t num_keys);
int x2g_keyed_row_sum(const float* src, const int32_t* key, int64_t rows, int32_t dim, int32_t num_keys,
                      float* out, int flags, void* workspace, size_t workspace_bytes, void* stream);

/* Several keyed row sums over the same keys (X2-GNN: every conv layer's per-destination edge
 * gradient summed into the element table's rows) as one partial launch + one slab-sum launch:
 * outs[j] (+)= keyed sum of srcs[j] (flags: X2G_ACCUM_WGRAD adds). */
#define X2G_KEYED_MAX_JOBS 8
size_t x2g_keyed_row_sum_batch_workspace(int64_t rows, int32_t dim, int32_t num_keys, int32_t num_jobs);
int x2g_keyed_row_sum_batch(const float* const* srcs, float* const* outs, int32_t num_jobs, const int32_t* key,
                            int64_t rows, int32_t dim, int32_t num_keys, int flags, void* workspace,
                            size_t workspace_bytes, void* stream);

/* PyG utils.softmax(src[R,H], index) for a sorted index (CSR rowptr): per segment and column,
 * exp(src - max) / (sum + 1e-16). */
int x2g_segment_softmax_fwd(const float* src, const int32_t* rowptr, int64_t num_segments, int64_t heads,
                            float* out, void* stream);
int x2g_segment_softmax_bwd(const float* out, const float* dout, const int32_t* rowptr,
                            int64_t num_segments, int64_t heads, float* dsrc, void* stream);

/* Index in ANY order (the operator-level drop-ins): the caller stable-sorts the keys on the device
 * and passes the permutation `perm` (sorted position r -> source row perm[r]) with the CSR row
 * pointer of the sorted keys; source rows are read in place through perm (no gathered copy).
 *   x2g_segment_reduce_perm: out[g] = sum (mode X2G_REDUCE_SUM) or mean (X2G_REDUCE_MEAN: / max(count,
 *     1), empty segments 0) of x[perm[r]], r in segment g — torch_scatter scatter_add / scatter_mean
 *     (readout.py:37,67-71; model.py:53), summed in the caller's row order;
 *   x2g_segment_reduce_perm_bwd: out[perm[r]] = g[seg(r)] (/ count for MEAN), its adjoint;
 *   x2g_segment_softmax_perm_fwd/bwd: PyG utils.softmax(src, index, num_nodes)
 *     (sbftransformer_conv.py:151) and its backward, written back in the caller's row order. */
#define X2G_REDUCE_SUM 0
#define X2G_REDUCE_MEAN 1
int x2g_segment_reduce_perm(const float* x, const int32_t* perm, const int32_t* rowptr, int64_t num_segments,
                            int64_t dim, int mode, float* out, void* stream);
int x2g_segment_reduce_perm_bwd(const float* g, const int32_t* perm, const int32_t* rowptr, int64_t num_segments,
                                int64_t dim, int mode, float* out, void* stream);
int x2g_segment_softmax_perm_fwd(const float* src, const int32_t* perm, const int32_t* rowptr,
                                 int64_t num_segments, int64_t heads, float* out, void* stream);
int x2g_segment_softmax_perm_bwd(const float* out, const float* dout, const int32_t* perm, const int32_t* rowptr,
                                 int64_t num_segments, int64_t heads, float* dsrc, void* stream);

/* PyG nn.LayerNorm(mode='graph', affine=False) (model.py:161,183): per segment g of rows,
 * mu = sum x / (n_g*D), var = sum (x-mu)^2 / (n_g*D) (n_g clamped >= 1), out = (x-mu)/sqrt(var+eps).
 * mean/rstd[num_segments] are saved for the backward. */
int x2g_graph_layernorm_fwd(const float* x, const int32_t* rowptr, int64_t num_segments, int64_t dim,
                            float eps, float* out, float* mean, float* rstd, void* stream);
int x2g_graph_layernorm_bwd(const float* out, const float* dout, const float* rstd, const int32_t* rowptr,
                            int64_t num_segments, int64_t dim, float* dx, void* stream);
/* The same backward with a workspace (x2g_graph_layernorm_bwd_workspace bytes): several workgroups
 * per segment, a stats pass and an apply pass (the segment's partial sums added in a fixed order). */
size_t x2g_graph_layernorm_bwd_workspace(int64_t num_segments);
int x2g_graph_layernorm_bwd_ex(const float* out, const float* dout, const float* rstd, const int32_t* rowptr,
                               int64_t num_segments, int64_t dim, float* dx, void* workspace, size_t workspace_bytes,
                               void* stream);
/* The same backward from per-row sums row_gstats[rows, 2] = (sum_c dout, sum_c dout * out) (as
 * x2g_chain_bwd_ln leaves them): one apply pass, no stats pass over dout and out. */
int x2g_graph_layernorm_bwd_rows(const float* out, const float* dout, const float* rstd, const int32_t* rowptr,
                                 int64_t num_segments, int64_t dim, const float* row_gstats, float* dx, void* stream);

/* ---------------------------------------------------------------- loss
 * F.smooth_l1_loss(pred, target, reduction='mean', beta) of the trainer step (trainer.py:41):
 * out[0] = mean over n of (|d| < beta ? 0.5 d^2 / beta : |d| - 0.5 beta), d = pred - target; the
 * backward dpred = gout[0] / n * clamp(d / beta, -1, 1).  One launch each way. */
int x2g_smooth_l1_mean_fwd(const float* pred, const float* target, int64_t n, float beta, float* out, void* stream);
int x2g_smooth_l1_mean_bwd(const float* pred, const float* target, int64_t n, float beta, const float* gout,
                           float* dpred, void* stream);
/* The forward that also writes dpred_unit = the backward's dpred for gout[0] = 1 (bit for bit): a
 * training step whose backward seed is 1 (trainer.py:42, loss.backward()) then needs no backward launch. */
int x2g_smooth_l1_mean_fwd_grad(const float* pred, const float* target, int64_t n, float beta, float* out,
                                float* dpred_unit, void* stream);

/* ---------------------------------------------------------------- dense-layer gradients */

/* Workspace bytes for x2g_linear_wgrad_ex (row-split partial slabs). */
size_t x2g_linear_wgrad_workspace(int64_t rows, int32_t out_features, int32_t in_features);


/* flags of the *_ex gradient entry points */
#define X2G_ACCUM_WGRAD 1 /* dw += ..., db += ... (write straight into a gradient buffer that already
                             holds a value, e.g. a zeroed flat all-reduce bucket) instead of dw = ... */
#define X2G_DEFER_SLAB_SUM 2 /* leave the per-workgroup weight-gradient partials in the workspace and
                                skip their fixed-order sum: the caller keeps the workspace alive and
                                sums many layers' partials in one x2g_slab_sum_batch launch */

/* One deferred weight-gradient reduction: dw[n_w] (+)= sum over `splits` slabs of part_w
 * (slab s at part_w + s*n_w), likewise db[n_b] from part_b (part_b/db may be NULL).
 * ld > 0: the slab is a [n_w / 128, 128] block of a larger weight: its row r lands at
 * dw + r * ld, first `cols` (<= 128) columns only (ld = 0: dw is the contiguous n_w block). */
typedef struct {
  const float* part_w;
  const float* part_b;
  float* dw;
  float* db;
  int64_t n_w;
  int32_t n_b;
  int32_t splits;
  int32_t ld;
  int32_t cols;
} x2g_slab_job;

/* Sum the slabs of njobs deferred reductions (host array of jobs) in as few launches as
 * possible; accum != 0: add into dw/db.  Same fixed order as the immediate sums. */
int x2g_slab_sum_batch(const x2g_slab_job* jobs, int32_t njobs, int32_t accum, void* stream);

/* Several readout pools over the same rows, segments and basis (X2-GNN's conv_layers + 1 AtomWise /
 * MolWise readouts all pool lin_rbf(rbf) * x_i edges -> atoms, readout.py:39-41,66-67) as ONE launch
 * each way instead of one per readout.  Forward uses x, w, b, out; backward g, x, w, b, dx, dx_add,
 * dw, db (meanings as x2g_rbf_gate_bwd / x2g_rbf_pool_fwd; owner maps rows to segments). */
#define X2G_GATE_MAX_JOBS 8
typedef struct {
  const float* x;      /* [rows, D] */
  const float* w;      /* lin_rbf weight [D, R] */
  const float* b;      /* [D] or NULL */
  float* out;          /* forward: pooled [n_seg, D] */
  const float* g;      /* backward: gradient of out (row r reads g[owner[r]]) */
  float* dx;           /* backward: [rows, D] or NULL */
  const float* dx_add; /* backward: added into dx (may alias it) or NULL */
  float* dw;           /* backward: [D, R] */
  float* db;           /* backward: [D] or NULL */
} x2g_gate_job;
int x2g_rbf_pool_fwd_batch(const x2g_gate_job* jobs, int32_t n_jobs, const float* rbf, const int32_t* rowptr,
                           int64_t n_seg, int32_t D, int32_t R, void* stream);
/* drbf (optional) receives the SUM of the jobs' basis gradients, in job order (X2G_GATE_DRBF_ACCUM:
 * added to it); dw / db as x2g_rbf_gate_bwd's flags, X2G_DEFER_SLAB_SUM returning one x2g_slab_job
 * per job in slab_jobs. */
size_t x2g_rbf_gate_bwd_batch_workspace(int64_t rows, int32_t D, int32_t R, int32_t n_jobs);
int x2g_rbf_gate_bwd_batch(const x2g_gate_job* jobs, int32_t n_jobs, const int32_t* owner, const float* rbf,
                           int64_t rows, int32_t D, int32_t R, float* drbf, int flags, x2g_slab_job* slab_jobs,
                           void* workspace, size_t workspace_bytes, void* stream);

/* Slab counts (and so the part_b offset, part_w + splits*n_w) of a deferred call. */
int32_t x2g_linear_wgrad_splits(int64_t rows, int32_t out_features, int32_t in_features);
int32_t x2g_dense_bwd_splits(int64_t rows, int32_t in_features, int32_t out_features);
/* Byte offset of those slabs inside x2g_dense_bwd_ex's workspace (part_w = workspace + offset;
 * x2g_linear_wgrad_ex's slabs start at its workspace). */
int64_t x2g_dense_bwd_slab_offset(int64_t rows, int32_t in_features, int32_t out_features);

/* dW[O,I] = dy[R,O]^T x[R,I] and db[O] = column sums of dy (db may be NULL): the weight/bias
 * gradient of every nn.Linear the reference applies row-wise (residual_layer.py, model.py:39,48,
 * readout.py, sbftransformer_conv.py:99-148, xgnn.py:54-70), split over rows with f32 MFMA and
 * summed in a fixed order (deterministic; replaces ATen's addmm backward through hipBLASLt);
 * flags X2G_ACCUM_WGRAD / X2G_DEFER_SLAB_SUM. */
int x2g_linear_wgrad_ex(const float* dy, const float* x, int64_t rows, int32_t out_features,
                        int32_t in_features, float* dw, float* db, int flags, void* workspace,
                        size_t workspace_bytes, void* stream);

#define X2G_ACT_NONE 0
#define X2G_ACT_SILU 1

/* Row-wise dense layer with fused epilogue: y[R,N] = act(x[R,K] w[N,K]^T + b[N]) (+ res[R,N]);
 * z[R,N] (optional) receives the pre-activation x w^T + b for the backward.  Replaces the
 * Linear -> SiLU -> add chains of residual_layer.py:21-27, model.py:39,47-50, readout.py:38-42,
 * xgnn.py:54-55,70 and the projections of sbftransformer_conv.py:99-107,127.  b, res, z may be NULL. */
int x2g_dense_fwd(const float* x, const float* w, const float* b, int64_t rows, int32_t in_features,
                  int32_t out_features, int act, const float* res, float* y, float* z, void* stream);

/* Workspace bytes for x2g_dense_bwd. */
size_t x2g_dense_bwd_workspace(int64_t rows, int32_t in_features, int32_t out_features);

/* Full backward of x2g_dense_fwd in one call: dz = dy * act'(z); dx = dz w (dx may be NULL: no
 * data gradient is formed); dw = dz^T x; db = colsum(dz) (db may be NULL).  For in/out features
 * <= 128 this is one persistent kernel (weight staged in LDS once per CU, dx and the per-CU
 * weight-gradient partials from the same LDS tiles) plus a fixed-order slab sum. */
int x2g_dense_bwd(const float* dy, const float* z, int act, const float* x, const float* w, int64_t rows,
                  int32_t in_features, int32_t out_features, float* dx, float* dw, float* db, void* workspace,
                  size_t workspace_bytes, void* stream);

/* x2g_dense_bwd plus: dx = dz w + dx_add (dx_add [R,K] optional, may alias dx: the gradient
 * contributions autograd would otherwise sum in a separate kernel — a residual branch, a tensor
 * feeding several layers) and flags (X2G_ACCUM_WGRAD: accumulate dw / db into their buffers).
 * Every shape supports dx_add (wider layers add it in the general kernel's epilogue). */
int x2g_dense_bwd_ex(const float* dy, const float* z, int act, const float* x, const float* w, int64_t rows,
                     int32_t in_features, int32_t out_features, float* dx, const float* dx_add, float* dw,
                     float* db, int flags, void* workspace, size_t workspace_bytes, void* stream);

/* ResidualLayer forward (residual_layer.py:21-27) in one persistent kernel:
 *   z0 = x w0^T + b0, h = SiLU(z0), z1 = h w1^T + b1, y = x + SiLU(z1)   (w0, w1: [D, D]; b optional)
 * h, z0, z1 are kept for the backward.  D <= 128, D % 4 == 0, 16-byte aligned rows
 * (X2G_EUNSUPPORTED otherwise). */
int x2g_residual_fwd(const float* x, const float* w0, const float* b0, const float* w1, const float* b1,
                     int64_t rows, int32_t dim, float* h, float* z0, float* z1, float* y, void* stream);

/* ---------------------------------------------------------------- batched layers (readout MLPs)
 * The trunk's conv_layers+1 readouts (model.py:41,50) run the same MLP shape on different inputs
 * with different weights: Linear(D,D)+SiLU, Linear(D,D)+SiLU, Linear(D,1) (readout.py:25-31,
 * 55-62), summed over readouts.  Each batched call runs G <= X2G_MAX_GROUPS of those layers in
 * one launch (blockIdx.y = group).  Supported: in/out features <= 128, multiples of 4, 16-byte
 * aligned rows (X2G_EUNSUPPORTED otherwise).  Group arrays are host memory, read at the call. */
#define X2G_MAX_GROUPS 8

typedef struct {
  const float* x;   /* [R, K] */
  const float* w;   /* [N, K] */
  const float* b;   /* [N] or NULL */
  const float* res; /* [R, N] or NULL */
  float* y;         /* [R, N] */
  float* z;         /* [R, N] pre-activation or NULL */
} x2g_dense_fwd_group;

typedef struct {
  const float* dy;     /* [R, N] */
  const float* z;      /* [R, N] (act == X2G_ACT_SILU) */
  const float* x;      /* [R, K] */
  const float* w;      /* [N, K] */
  float* dx;           /* [R, K] or NULL */
  const float* dx_add; /* [R, K] or NULL */
  float* dw;           /* [N, K] */
  float* db;           /* [N] or NULL */
} x2g_dense_bwd_group;

int x2g_dense_fwd_batched(const x2g_dense_fwd_group* groups, int32_t num_groups, int64_t rows,
                          int32_t in_features, int32_t out_features, int act, void* stream);

/* Workspace: num_groups * x2g_dense_bwd_workspace(rows, K, N); group g's weight-gradient slabs
 * (x2g_dense_bwd_splits of them) start at byte g * x2g_dense_bwd_workspace(rows, K, N).  Flags as
 * x2g_dense_bwd_ex; without X2G_DEFER_SLAB_SUM one x2g_slab_sum_batch launch sums all groups. */
int x2g_dense_bwd_batched(const x2g_dense_bwd_group* groups, int32_t num_groups, int64_t rows,
                          int32_t in_features, int32_t out_features, int act, int flags, void* workspace,
                          size_t workspace_bytes, void* stream);

/* The readouts' last Linear(D, 1) summed over groups: out[r] = sum_g (h_g[r, :] . w_g + b_g). */
typedef struct {
  const float* h; /* [R, D] */
  const float* w; /* [D] */
  const float* b; /* [1] or NULL */
  float* dh;      /* backward: [R, D] = dout[r] * w_g (NULL: not needed) */
  float* dw;      /* backward: [D] */
  float* db;      /* backward: [1] or NULL */
} x2g_head_group;

int x2g_readout_head_fwd(const x2g_head_group* groups, int32_t num_groups, int64_t rows, int32_t dim, float* out,
                         void* stream);
size_t x2g_readout_head_bwd_workspace(int64_t rows, int32_t dim, int32_t num_groups);
int32_t x2g_readout_head_bwd_splits(int64_t rows);
/* dh_g = dout w_g^T, dw_g (+)= sum_r dout[r] h_g[r], db_g (+)= sum_r dout[r]; flags as
 * x2g_linear_wgrad_ex (group g's slabs: splits*dim floats at g*splits*(dim+1) floats into the
 * workspace, then its bias slabs: splits floats). */
int x2g_readout_head_bwd(const float* dout, const x2g_head_group* groups, int32_t num_groups, int64_t rows,
                         int32_t dim, int flags, void* workspace, size_t workspace_bytes, void* stream);

/* The heads with the per-molecule sum fused (AtomWise's per-atom outputs pooled by the global add pool,
 * model.py:53): out_seg[m] = sum over rows r of segment m (seg_rowptr[m] .. seg_rowptr[m+1]) of
 * sum_g (h_g[r] . w_g + b_g); and the backward from d out_seg (dh_g[r] = dout_seg[seg(r)] w_g, dw_g / db_g as
 * x2g_readout_head_bwd, same workspace).  One launch each way instead of head + pool / broadcast + head. */
int x2g_readout_head_pool_fwd(const x2g_head_group* groups, int32_t num_groups, int64_t rows, int32_t dim,
                              const int32_t* seg_rowptr, int64_t num_segments, float* out_seg, void* stream);
int x2g_readout_head_pool_bwd(const float* dout_seg, const int32_t* seg_rowptr, int64_t num_segments,
                              const x2g_head_group* groups, int32_t num_groups, int64_t rows, int32_t dim, int flags,
                              void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- parameter update */

/* float[16] device scalar block of x2g_clip_adam_ema: the caller sets the hyper-parameters,
 * the library maintains the rest (so a captured HIP graph replays correct steps). */
#define X2G_OPT_LR 0
#define X2G_OPT_BETA1 1
#define X2G_OPT_BETA2 2
#define X2G_OPT_EPS 3
#define X2G_OPT_MAX_NORM 4  /* <= 0: no clipping */
#define X2G_OPT_EMA_DECAY 5
#define X2G_OPT_STEP 6      /* steps taken (float); incremented by every call */
#define X2G_OPT_NORM 7      /* out: total gradient 2-norm before clipping */
#define X2G_OPT_CLIP 8      /* out: clip coefficient applied */
#define X2G_OPT_STEP_SIZE 9 /* internal: lr / (1 - beta1^t) */
#define X2G_OPT_BC2_SQRT 10 /* internal: sqrt(1 - beta2^t) */
/* Optional on-device LR schedule, LinearWarmupExponentialDecay (scheduler.py:4-31; config.json
 * warmup_steps 3000, decay_steps 3e6, decay_rate 0.01), evaluated from the device step count so a
 * captured graph follows it: when X2G_OPT_WARMUP > 0, step t (0-based, the steps taken before it)
 * uses lr = BASE_LR * min(1/W + t/W, 1) * DECAY_RATE^(t / DECAY_STEPS) (the exponent floored with
 * STAIRCASE != 0), computed in double as LambdaLR does, and the value used is left in X2G_OPT_LR. */
#define X2G_OPT_WARMUP 11
#define X2G_OPT_DECAY_STEPS 12
#define X2G_OPT_DECAY_RATE 13
#define X2G_OPT_BASE_LR 14
#define X2G_OPT_STAIRCASE 15

/* Workspace bytes for x2g_clip_adam_ema. */
size_t x2g_optimizer_workspace(int64_t n);

/* The reference trainer's update (trainer.py:43-48, train_ema.py:45-48) over one flat fp32
 * parameter buffer of n elements: clip_grad_norm_(max_norm) (coef = max_norm/(norm+1e-6),
 * clamped to 1), torch.optim.Adam (amsgrad=False, no weight decay), then the EMA
 * ema = d*ema + (1-d)*p (ema may be NULL; at step 1 ema = p, as AveragedModel's first
 * update_parameters copies).  grads must be 16-byte aligned; the gradient
 * buffer is read, not modified.  Deterministic (fixed-order norm reduction). */
int x2g_clip_adam_ema(float* params, const float* grads, float* exp_avg, float* exp_avg_sq, float* ema,
                      int64_t n, float* scalars, void* workspace, size_t workspace_bytes, void* stream);
/* x2g_clip_adam_ema with flags: X2G_OPT_ZERO_GRADS zeroes each gradient element once the update
 * has read it (optimizer.zero_grad() folded into the step: the next backward may accumulate into
 * the buffer without a separate fill). */
#define X2G_OPT_ZERO_GRADS 1
int x2g_clip_adam_ema_ex(float* params, float* grads, float* exp_avg, float* exp_avg_sq, float* ema, int64_t n,
                         float* scalars, int flags, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- row chains (trunk tail)
 *
 * One conv layer of the trunk ends in seven row-wise Linear layers on the same E rows
 * (model.py:47-50): bf_skip = ResidualLayer (2 Linear), SiLU(dense_bf_skip(.)) + the conv
 * input, af_skip = 2 x ResidualLayer (4 Linear).  A "chain" runs such a sequence of D x D
 * stages in ONE kernel with every 16-row tile held in registers from the first stage to the
 * last (the stage weights stream through LDS), so the chain pays one launch and one pipeline
 * ramp instead of seven.  Stage s:  z_s = in_s W_s^T + b_s,  out_s = act_s(z_s) (+ residual),
 * in_{s+1} = out_s.  Compiled for D = 128 (X2G_EUNSUPPORTED otherwise), rows * 128 < 2^31,
 * 16-byte aligned row-major [rows, 128] tensors. */
#define X2G_CHAIN_MAX_STAGES 8
#define X2G_CHAIN_SILU 1     /* act_s = SiLU (else identity) */
#define X2G_CHAIN_HOLD 2     /* in_s becomes the held residual (the input of a ResidualLayer) */
#define X2G_CHAIN_RES_HELD 4 /* out_s += the held residual */
#define X2G_CHAIN_RES_EXT 8  /* out_s += res_ext (at most one stage; a HOLD .. RES_HELD pair must
                                not span it, and a stage adds one residual at most) */
#define X2G_CHAIN_RES_ACCUM 16 /* backward only, with RES_EXT: d_res_ext += (instead of =) the
                                  residual's gradient (res_ext feeds other layers too) */

typedef struct {
  const float* w; /* [D, D] nn.Linear weight, row n = output feature n */
  const float* b; /* [D] or NULL */
  float* z;       /* [rows, D] pre-activation out (kept for the backward), or NULL */
  float* y;       /* [rows, D] stage output out (the next stage's input); required for the last stage */
  float* wt;      /* [D, D] out: w transposed, for x2g_chain_bwd (NULL: not written) */
  int32_t flags;
} x2g_chain_stage;

/* Forward of a chain of n_stages (1..X2G_CHAIN_MAX_STAGES) stages on x [rows, dim].
 * in_t (optional): every stage's input (x, then each stage's output) in the tiled-transposed layout
 * below, stage s at in_t + s * x2g_chain_t_floats(rows, dim) — the operand x2g_chain_wgrad reads. */
int x2g_chain_fwd(const float* x, const float* res_ext, const x2g_chain_stage* stages, int32_t n_stages,
                  int64_t rows, int32_t dim, float* in_t, void* stream);

/* x2g_chain_fwd on LayerNorm(x): the chain's input is PyG's graph LayerNorm of x (model.py:46,
 * mode='graph', affine=False: per segment g = rows [seg_rowptr[g], seg_rowptr[g+1]) of the
 * num_segments molecules covering all rows, out = (x - mean_g) / sqrt(var_g + eps) over every row
 * and feature of the segment), computed while the input is staged from row_stats [rows, 2] (the
 * (mean, M2) per row of x2g_sbf_attention_fwd_stats): no separate LayerNorm pass.  Also writes the
 * normalised rows x_norm [rows, dim] (or NULL) and seg_mean / seg_rstd [num_segments] (or NULL) —
 * the inputs of x2g_graph_layernorm_bwd_ex, which completes the backward.  The stage weight
 * gradients see the normalised rows as the chain's input (in_t). */
int x2g_chain_fwd_ln(const float* x, const float* row_stats, const int32_t* seg_rowptr, int64_t num_segments,
                     float eps, float* x_norm, float* seg_mean, float* seg_rstd, const float* res_ext,
                     const x2g_chain_stage* stages, int32_t n_stages, int64_t rows, int32_t dim, float* in_t,
                     void* stream);

/* Several independent chains over the same row count and stage count in ONE launch (job =
 * blockIdx.y; X2-GNN's readout MLPs, readout.py:25-31 / 55-62: Linear+SiLU, Linear+SiLU on the
 * pooled atom rows of every readout).  Each job's fields mean what x2g_chain_fwd's / _bwd's do. */
#define X2G_CHAIN_MAX_JOBS 8
typedef struct {
  const float* x;
  const float* res_ext;
  const x2g_chain_stage* stages; /* n_stages */
  float* in_t;
} x2g_chain_fwd_job;
int x2g_chain_fwd_batch(const x2g_chain_fwd_job* jobs, int32_t num_jobs, int32_t n_stages, int64_t rows, int32_t dim,
                        void* stream);

/* Tiled-transposed ("T") layout of a [rows, D] tensor: 16-row tiles; tile t holds element (r, f)
 * at t*16*D + f*16 + (r - 16t), rows past `rows` in the last tile zero.  Floats per tensor: */
int64_t x2g_chain_t_floats(int64_t rows, int32_t dim);

typedef struct {
  const float* w; /* [D, D] the stage's weight */
  const float* wt; /* [D, D] w transposed (x2g_chain_fwd's wt output), or NULL: w is read transposed */
  const float* z; /* [rows, D] its saved pre-activation (required for SiLU stages) */
  float* dz;      /* [rows, D] out: dL/dz_s (the input of the stage's weight gradient) */
  int32_t flags;  /* the forward's flags */
} x2g_chain_bwd_stage;

/* Data gradients of x2g_chain_fwd: dy (+ dy_add, may be NULL) = dL/d out_{n-1}; writes every
 * stage's dz (row-major where the stage's dz is set; T layout at dz_t + s * x2g_chain_t_floats when
 * dz_t is set), dx = dL/dx and d_res_ext = dL/d res_ext (NULL when no stage has RES_EXT).
 * Weight gradients: x2g_chain_wgrad over (in_t, dz_t), or x2g_wgrad_batched over row-major pairs. */
int x2g_chain_bwd(const float* dy, const float* dy_add, const x2g_chain_bwd_stage* stages, int32_t n_stages,
                  int64_t rows, int32_t dim, float* dx, float* d_res_ext, float* dz_t, void* stream);
/* x2g_chain_bwd for a chain run by x2g_chain_fwd_ln: also writes row_gstats[rows, 2] = (sum_c dx,
 * sum_c dx * x_norm) per row, the input of x2g_graph_layernorm_bwd_rows (x_norm: x2g_chain_fwd_ln's). */
int x2g_chain_bwd_ln(const float* dy, const float* dy_add, const x2g_chain_bwd_stage* stages, int32_t n_stages,
                     int64_t rows, int32_t dim, float* dx, float* d_res_ext, float* dz_t, const float* x_norm,
                     float* row_gstats, void* stream);

/* x2g_chain_bwd for several chains (x2g_chain_fwd_batch's jobs) in one launch. */
typedef struct {
  const float* dy;
  const float* dy_add;
  const x2g_chain_bwd_stage* stages; /* n_stages */
  float* dx;
  float* d_res_ext;
  float* dz_t;
} x2g_chain_bwd_job;
int x2g_chain_bwd_batch(const x2g_chain_bwd_job* jobs, int32_t num_jobs, int32_t n_stages, int64_t rows, int32_t dim,
                        void* stream);

/* Weight / bias gradients of every chain stage: dw[s] = dz_s^T in_s, db[s] = colsum(dz_s) (db[s] may
 * be NULL) from the T-layout operands of x2g_chain_fwd / x2g_chain_bwd; dw / db are host arrays of
 * n_stages device pointers.  Rows are split into fixed tile ranges per stage, the partials summed
 * in a fixed order; flags and slab layout as x2g_wgrad_batched (stage s's slabs at byte
 * s * (workspace / n_stages)). */
size_t x2g_chain_wgrad_workspace(int64_t rows, int32_t dim, int32_t n_stages);
int x2g_chain_wgrad(const float* in_t, const float* dz_t, int32_t n_stages, int64_t rows, int32_t dim,
                    float* const* dw, float* const* db, int flags, void* workspace, size_t workspace_bytes,
                    void* stream);

/* Weight / bias gradients of up to X2G_CHAIN_MAX_STAGES independent D x D Linear layers over the
 * same rows: dw_g = dy_g^T x_g, db_g = column sums of dy_g (db_g may be NULL).  Rows are split
 * into fixed chunks per layer (one workgroup each, f32 MFMA), chunk partials summed in a fixed
 * order (deterministic); flags X2G_ACCUM_WGRAD / X2G_DEFER_SLAB_SUM as x2g_linear_wgrad_ex.  Layer
 * g's slabs: x2g_wgrad_batched_splits() slabs of D*D floats starting at byte g * (workspace(rows,
 * dim, num_jobs) / num_jobs), then its bias slabs (D floats each). */
typedef struct {
  const float* dy; /* [rows, D] */
  const float* x;  /* [rows, D] */
  float* dw;       /* [D, D] */
  float* db;       /* [D] or NULL */
} x2g_wgrad_job;

size_t x2g_wgrad_batched_workspace(int64_t rows, int32_t dim, int32_t num_jobs);
int32_t x2g_wgrad_batched_splits(int64_t rows, int32_t dim, int32_t num_jobs);
int x2g_wgrad_batched(const x2g_wgrad_job* jobs, int32_t num_jobs, int64_t rows, int32_t dim, int flags,
                      void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- conv projections
 * The five projections SBFTransformerConv.forward applies to its node features
 * (sbftransformer_conv.py:99-107,127): f = lin_rbf(rbf) (no bias), x_src = x * f,
 * q = lin_query(x), k = lin_key(x_src), v = lin_value(x_src), skip = lin_skip(x) — one kernel with
 * each CU's rows of x and x_src held in LDS (the row-chain v2 structure), D = 128, rbf_dim <= 8.
 * proj[0..3] = query, key, value, skip: w [D, D], b [D] or NULL, out [rows, D], wt (optional out:
 * w transposed, for the backward).  x_t / xs_t (optional): x and x_src in the T layout (the
 * weight gradient's operands).  */
typedef struct {
  const float* w;
  const float* b;
  float* out;
  float* wt;
} x2g_proj;

int x2g_conv_proj_fwd(const float* x, const float* rbf, int32_t rbf_dim, const float* w_rbf, const x2g_proj* proj,
                      int64_t rows, int32_t dim, float* x_t, float* xs_t, void* stream);

/* The gradients x2g_conv_proj_fwd's backward takes: grads[0..3] = dL/d(q, k, v, skip) with their
 * weights (w, or wt when given) and optional T-layout copies g_t for the weight gradient
 * (x2g_tiled_wgrad):  dx = dq Wq + dskip Ws (+ dx_add; dx may alias dx_add),  dxs = dk Wk + dv Wv
 * = dL/d x_src. */
typedef struct {
  const float* g;
  const float* w;
  const float* wt;
  float* g_t;
} x2g_proj_grad;

/* The projections' data gradient with the gate's backward folded in, dxs kept in
 * registers: dx = dq Wq + dskip Ws (+ dx_add) + dxs * f with f = rbf W_rbf^T; drbf (optional,
 * [rows, rbf_dim]) = (dxs * x) W_rbf, added to its contents with X2G_GATE_DRBF_ACCUM; dw_rbf
 * [dim, rbf_dim] (+)= (dxs * x)^T rbf from one slab per workgroup (flags X2G_ACCUM_WGRAD,
 * X2G_DEFER_SLAB_SUM: x2g_conv_proj_bwd_gate_splits slabs of dim*rbf_dim floats at the workspace,
 * no part_b).  Replaces sbftransformer_conv.py:99-100's backward (x_src = x * lin_rbf(rbf)). */
int32_t x2g_conv_proj_bwd_gate_splits(int64_t rows);
size_t x2g_conv_proj_bwd_gate_workspace(int64_t rows, int32_t rbf_dim);
int x2g_conv_proj_bwd_gate(const x2g_proj_grad* grads, int64_t rows, int32_t dim, const float* x, const float* rbf,
                           int32_t rbf_dim, const float* w_rbf, float* dx, const float* dx_add, float* drbf,
                           float* dw_rbf, int flags, void* workspace, size_t workspace_bytes, void* stream);

/* Weight / bias gradients of independent D x D Linear layers over the same rows from T-layout
 * operands: dw_j = dy_j^T x_j, db_j = colsum(dy_j) (db_j may be NULL); as x2g_chain_wgrad, with
 * each job's operands given separately (a T-layout tensor may serve several jobs). */
typedef struct {
  const float* dy_t;
  const float* x_t;
  float* dw;
  float* db;
  int32_t ld;   /* 0: dw is a [D, D] weight; > 0: dw is the top-left of a D x D block of a larger */
  int32_t cols; /* weight with row stride ld, of which the first `cols` (<= D) columns are written */
} x2g_tiled_job;

/* The same for up to X2G_TILED_MAX_JOBS jobs (e.g. every T-layout weight gradient of a backward)
 * in ONE launch: the jobs' 16-row tiles are concatenated and split evenly over one workgroup per
 * CU, so a job's partials are the few workgroups overlapping it (~256 + num_jobs slabs in all).
 * With X2G_DEFER_SLAB_SUM the num_jobs slab reductions are returned in slab_jobs (host array) for
 * the caller's x2g_slab_sum_batch; otherwise they are summed here. */
#define X2G_TILED_MAX_JOBS 64
size_t x2g_tiled_wgrad_flat_workspace(int64_t rows, int32_t dim, int32_t num_jobs);
int x2g_tiled_wgrad_flat(const x2g_tiled_job* jobs, int32_t num_jobs, int64_t rows, int32_t dim, int flags,
                         x2g_slab_job* slab_jobs, void* workspace, size_t workspace_bytes, void* stream);
/* The same with a row count per job (job_rows: HOST array of num_jobs): a backward's weight gradients
 * over the line-node rows and over the atom rows (the readout MLPs) in one launch instead of one per
 * row count.  Equal row counts reproduce x2g_tiled_wgrad_flat exactly. */
size_t x2g_tiled_wgrad_flat_rows_workspace(const int64_t* job_rows, int32_t num_jobs, int32_t dim);
int x2g_tiled_wgrad_flat_rows(const x2g_tiled_job* jobs, const int64_t* job_rows, int32_t num_jobs, int32_t dim,
                              int flags, x2g_slab_job* slab_jobs, void* workspace, size_t workspace_bytes,
                              void* stream);

size_t x2g_tiled_wgrad_workspace(int64_t rows, int32_t dim, int32_t num_jobs);
int x2g_tiled_wgrad(const x2g_tiled_job* jobs, int32_t num_jobs, int64_t rows, int32_t dim, int flags,
                    void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- small-table chains
 * X2-GNN's edge attribute is the embedding of the middle atom (xgnn.py:57-58), so the embedding
 * Linear (atom_embedding.py:22-25), edgenn (model.py:39) and every conv layer's lin_edge
 * (sbftransformer_conv.py:144) act on the per-element table.  Those layers form a tree of D x D
 * Linear stages on <= 16 rows: stage s reads x (parent -1) or the output of an earlier stage,
 *     z_s = in_s W_s^T + b_s,   y_s = act_s(z_s).
 * One workgroup runs the whole tree per direction (one launch instead of one GEMM per layer).
 * D = 128, rows <= 16 (X2G_EUNSUPPORTED otherwise), 16-byte aligned weights / rows. */
#define X2G_TABLE_MAX_STAGES 8

typedef struct {
  const float* w; /* [D, D] nn.Linear weight */
  const float* b; /* [D] or NULL */
  int32_t parent; /* -1: x, else an earlier stage (< s) */
  int32_t act;    /* 0 identity, 1 SiLU */
  float* z;       /* [rows, D] out: pre-activation (required when act = SiLU), or NULL */
  float* y;       /* [rows, D] out: the stage output */
} x2g_table_stage;

int x2g_table_chain_fwd(const float* x, int64_t rows, int32_t dim, const x2g_table_stage* stages, int32_t n_stages,
                        void* stream);

typedef struct {
  const float* w;  /* [D, D] the stage's weight */
  const float* in; /* [rows, D] the stage's forward input (x or the parent's y) */
  const float* z;  /* [rows, D] saved pre-activation (SiLU stages) */
  const float* dy; /* [rows, D] dL/dy_s from outside the tree, or NULL (children's shares are added in) */
  float* dw;       /* [D, D] out: dL/dW_s */
  float* db;       /* [D] out: dL/db_s, or NULL */
  int32_t parent;
  int32_t act;
  int32_t accum;   /* 1: dw / db += the gradient (a gradient bucket), 0: overwrite */
} x2g_table_bwd_stage;

/* Backward of x2g_table_chain_fwd (stages in the forward's order): every stage's weight / bias
 * gradient and dx = dL/dx ([rows, D], may be NULL), with a workspace (x2g_table_chain_bwd_workspace
 * bytes, 16-byte aligned; it receives every stage's dz): two launches — the dz / dx chain through the
 * tree in one workgroup (children before parents), then every stage's dW / db side by side, one
 * workgroup each.  The forward runs one workgroup per root-to-leaf path. */
size_t x2g_table_chain_bwd_workspace(int32_t n_stages);
int x2g_table_chain_bwd_ex(const x2g_table_bwd_stage* stages, int32_t n_stages, int64_t rows, int32_t dim, float* dx,
                           void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- line-node featurisation
 * neo_x = SiLU(emb_trans(SiLU(mat_trans(x * env))))  (xgnn.py:49-56 of the reference: mat_trans
 * 338 -> 256, emb_trans 256 -> 128, x the per-line-node input features, env the envelope).
 * Forward in one kernel: y [rows, 128] plus the backward's operands in the T layout above with
 * 128-feature planes (plane p at +p * x2g_chain_t_floats(rows, 128)): xs_t = x * env (3 planes,
 * features past in_dim zero), z1_t / y1_t = mat_trans pre-activation / output (2 planes),
 * z2_t = emb_trans pre-activation (1 plane).  Compiled for 256 < in_dim <= 384, in_dim even; w1
 * [256, in_dim] 8-byte aligned, w2 [128, 256]; env may be NULL (1). */
int x2g_feat_fwd(const float* x, const float* env, int64_t rows, int32_t in_dim, const float* w1, const float* b1,
                 const float* w2, const float* b2, float* y, float* xs_t, float* z1_t, float* y1_t, float* z2_t,
                 void* stream);

/* Data part of the backward: dz2_t = dy SiLU'(z2), dz1_t = (dz2 W2) SiLU'(z1), T layout (1 and 2
 * planes).  The weight gradients are x2g_tiled_wgrad jobs: dW1 block (o, i) = dz1_t plane o x
 * xs_t plane i (ld = in_dim, cols = min(128, in_dim - 128 i)), dW2 block i = dz2_t x y1_t plane i. */
int x2g_feat_bwd(const float* dy, const float* z2_t, const float* z1_t, const float* w2, int64_t rows, float* dz2_t,
                 float* dz1_t, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* X2G_H */
