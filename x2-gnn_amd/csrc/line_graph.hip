// Line-graph (triplet) construction on the device.
//
// Replaces vertex_to_edge_2 (edge_graph.py:12-30), which the reference runs on the CPU with
// scipy on every forward (xgnn.py:52-53: a D2H copy of edge_index, scipy CSR slicing, an H2D
// copy of the triplets).  Here it is count -> exclusive scan -> emit, all integer work, with
// sizes from host metadata so nothing is read back.
//
// Ordering contract (the reference's): triplets are grouped by destination line node
// e=(a->b) in edge order, and inside a group k ascends (scipy CSR rows are column-sorted).
// With edges sorted by (src, dst) -- np.argwhere order, atom_graph.py:42-45 -- the edges out
// of atom b are the contiguous range atom_rowptr[b]..atom_rowptr[b+1] in ascending k, and the
// id of edge (b->k) is its position in that range.
#include <algorithm>
#include <numeric>
#include <vector>

#include "common.hpp"

namespace x2g {

// ----------------------------------------------------------------------------- CSR row ptr
__global__ void rowptr_kernel(const int32_t* __restrict__ keys, int64_t n, int64_t n_seg,
                              int32_t* __restrict__ rowptr) {
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i > n) return;
  int64_t prev = (i == 0) ? -1 : keys[i - 1];
  int64_t cur = (i == n) ? n_seg : keys[i];
  if (prev < -1) prev = -1;  // out-of-range keys never write outside rowptr
  if (cur > n_seg) cur = n_seg;
  for (int64_t s = prev + 1; s <= cur; ++s) rowptr[s] = static_cast<int32_t>(i);
}

// rowptr[s] = lower_bound(keys, s) for s in [0, n_seg] (binary search: every entry written, always in
// [0, n]); threads i < n also check the keys' contract and flag a violation with a plain vector store
// of 1 (every writer stores the same value, so the race is benign; no atomics).
__global__ void rowptr_checked_kernel(const int32_t* __restrict__ keys, int64_t n, int64_t n_seg,
                                      int32_t* __restrict__ rowptr, int32_t* __restrict__ status) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i <= n_seg) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (keys[mid] < i) lo = mid + 1;
      else hi = mid;
    }
    rowptr[i] = static_cast<int32_t>(lo);
  }
  if (i < n) {
    const int32_t k = keys[i];
    if (k < 0 || k >= n_seg || (i > 0 && keys[i - 1] > k)) status[0] = 1;
  }
}

// ----------------------------------------------------------------------------- exclusive scan
// Three-phase scan of int32 counts: 1024 elements per 256-thread block, block totals scanned
// by one block, then offsets added.  out has n+1 entries (out[n] = total).
constexpr int kScanThreads = 256;
constexpr int kScanPerThread = 4;
constexpr int kScanTile = kScanThreads * kScanPerThread;

__device__ __forceinline__ int block_exclusive_scan(int v, int* lds_wave, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    int y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) lds_wave[wave] = incl;
  __syncthreads();
  int wave_off = 0, tot = 0;
  const int nw = blockDim.x >> 6;
  for (int w = 0; w < nw; ++w) {
    int s = lds_wave[w];
    if (w < wave) wave_off += s;
    tot += s;
  }
  *total = tot;
  __syncthreads();
  return wave_off + incl - v;
}

__global__ void __launch_bounds__(kScanThreads) scan_tiles(const int32_t* __restrict__ in, int64_t n,
                                                           int32_t* __restrict__ out,
                                                           int32_t* __restrict__ partial) {
  __shared__ int lds[kScanThreads / 64];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile + threadIdx.x * kScanPerThread;
  int v[kScanPerThread];
  int sum = 0;
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    v[i] = (base + i < n) ? in[base + i] : 0;
    sum += v[i];
  }
  int total;
  int run = block_exclusive_scan(sum, lds, &total);
#pragma unroll
  for (int i = 0; i < kScanPerThread; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = total;
}

// One block: exclusive scan of the tile totals in place; partial[nb] = grand total.
__global__ void __launch_bounds__(1024) scan_partials(int32_t* __restrict__ partial, int64_t nb) {
  __shared__ int lds[1024 / 64];
  int carry = 0;
  for (int64_t c = 0; c < nb; c += blockDim.x) {
    int64_t i = c + threadIdx.x;
    int v = (i < nb) ? partial[i] : 0;
    int total;
    int ex = block_exclusive_scan(v, lds, &total);
    if (i < nb) partial[i] = carry + ex;
    carry += total;
  }
  if (threadIdx.x == 0) partial[nb] = carry;
}

__global__ void scan_add(int32_t* __restrict__ out, int64_t n, const int32_t* __restrict__ partial,
                         int64_t nb) {
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kScanTile;
  const int off = partial[blockIdx.x];
  for (int i = threadIdx.x; i < kScanTile; i += blockDim.x)
    if (base + i < n) out[base + i] += off;
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = partial[nb];
}

inline int64_t scan_partials_ints(int64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

int exclusive_scan(const int32_t* in, int64_t n, int32_t* out, int32_t* partial, hipStream_t st) {
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb == 0) {
    const hipError_t e = hipMemsetAsync(out, 0, sizeof(int32_t), st);
    return e == hipSuccess ? X2G_OK : static_cast<int>(e);
  }
  scan_tiles<<<static_cast<unsigned>(nb), kScanThreads, 0, st>>>(in, n, out, partial);
  scan_partials<<<1, 1024, 0, st>>>(partial, nb);
  scan_add<<<static_cast<unsigned>(nb), kScanThreads, 0, st>>>(out, n, partial, nb);
  return last_launch_status();
}

// ----------------------------------------------------------------------------- triplets
__device__ __forceinline__ int lower_bound(const int32_t* __restrict__ a, int lo, int hi, int key) {
  while (lo < hi) {
    int mid = (lo + hi) >> 1;
    if (a[mid] < key) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// count[e] = |N_out(b) \ {a}| for e = (a->b)
__global__ void triplet_count_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                     const int32_t* __restrict__ atom_rowptr, int64_t E,
                                     int32_t* __restrict__ count) {
  int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int a = src[e], b = dst[e];
  const int lo = atom_rowptr[b], hi = atom_rowptr[b + 1];
  const int p = lower_bound(dst, lo, hi, a);
  const int has_rev = (p < hi && dst[p] == a) ? 1 : 0;
  count[e] = hi - lo - has_rev;
}

// Emit the triplets of 8 destination edges per wave: lane group of 8 walks N_out(b) in
// chunks of 8, compacts with a ballot so writes of one group are contiguous.
constexpr int kEmitGroup = 8;
__device__ __forceinline__ void emit_group(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                           const int32_t* __restrict__ atom_rowptr,
                                           const int32_t* __restrict__ trip_rowptr, int64_t E, int64_t T,
                                           int32_t* __restrict__ trip_src, int32_t* __restrict__ trip_dst,
                                           int32_t* __restrict__ atom_j, int32_t* __restrict__ atom_i,
                                           int32_t* __restrict__ atom_k, int32_t* __restrict__ edge_rev = nullptr,
                                           int32_t* __restrict__ rev_trip = nullptr) {
  const int64_t gtid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t e = gtid / kEmitGroup;
  const int sub = threadIdx.x & (kEmitGroup - 1);
  const int lane = threadIdx.x & 63;
  const uint64_t group_mask = ((1ull << kEmitGroup) - 1) << (lane & ~(kEmitGroup - 1));
  const bool valid = e < E;
  int a = 0, b = 0, lo = 0, hi = 0, p = 0;
  if (valid) {
    a = src[e];
    b = dst[e];
    lo = atom_rowptr[b];
    hi = atom_rowptr[b + 1];
    p = trip_rowptr[e];
  }
  const int p0 = p;
  // loop until every group in the wave is done (wave-uniform trip count via __any)
  for (int base = lo; __any(valid && base < hi); base += kEmitGroup) {
    const int idx = base + sub;
    const bool in = valid && idx < hi;
    const int k = in ? dst[idx] : -1;
    const bool keep = in && k != a;
    // the excluded neighbour k == a is the reverse edge b->a: for the center-atom attention kernels,
    // edge_rev[e] = id(b->a) and rev_trip[b->a] = trip_rowptr[e] (symmetric graphs: every edge has one)
    if (edge_rev && in && k == a) {
      edge_rev[e] = idx;
      rev_trip[idx] = p0;
    }
    const uint64_t ball = __ballot(keep) & group_mask;
    const uint64_t below = ball & ((1ull << lane) - 1);
    const int q = p + __popcll(below);
    if (keep && q < T) {  // q >= T only if the host-provided T is too small: never write past it
      trip_src[q] = idx;
      trip_dst[q] = static_cast<int32_t>(e);
      if (atom_j) atom_j[q] = b;
      if (atom_i) atom_i[q] = a;
      if (atom_k) atom_k[q] = k;
    }
    p += __popcll(ball);
  }
}

__global__ void triplet_emit_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                    const int32_t* __restrict__ atom_rowptr,
                                    const int32_t* __restrict__ trip_rowptr, int64_t E, int64_t T,
                                    int32_t* __restrict__ trip_src, int32_t* __restrict__ trip_dst,
                                    int32_t* __restrict__ atom_j, int32_t* __restrict__ atom_i,
                                    int32_t* __restrict__ atom_k, int32_t* __restrict__ edge_rev,
                                    int32_t* __restrict__ rev_trip) {
  emit_group(src, dst, atom_rowptr, trip_rowptr, E, T, trip_src, trip_dst, atom_j, atom_i, atom_k, edge_rev, rev_trip);
}

// ----------------------------------------------------------------------------- transpose
__global__ void count_by_key(const int32_t* __restrict__ keys, int64_t n, int32_t* __restrict__ count) {
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) atomicAdd(&count[keys[i]], 1);
}

__global__ void fill_by_key(const int32_t* __restrict__ keys, int64_t n, const int32_t* __restrict__ rowptr,
                            int32_t* __restrict__ cursor, int32_t* __restrict__ perm) {
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int s = keys[i];
  const int pos = atomicAdd(&cursor[s], 1);
  perm[rowptr[s] + pos] = static_cast<int32_t>(i);
}

// The atomic fill leaves each segment in arrival order; sort it (segments are short:
// the in-degree of one atom) so the result, and every float sum over it, is deterministic.
__global__ void sort_segments(const int32_t* __restrict__ rowptr, int64_t n_seg, int32_t* __restrict__ perm) {
  int64_t s = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (s >= n_seg) return;
  const int lo = rowptr[s], hi = rowptr[s + 1];
  for (int i = lo + 1; i < hi; ++i) {
    const int v = perm[i];
    int j = i - 1;
    while (j >= lo && perm[j] > v) {
      perm[j + 1] = perm[j];
      --j;
    }
    perm[j + 1] = v;
  }
}


// ----------------------------------------------------------------------------- symmetric graphs
// A molecule's edge set is symmetric (a->b present iff b->a is, atom_graph.py:42-45 builds it from
// a symmetric distance test), which makes both per-edge counts a degree: destination e = (a->b)
// has deg(b) - 1 triplets (b->a is the one excluded) and source s = (b->k) feeds deg(b) - 1
// destinations (a->b), a != k.  Counting needs no search, so count and scan are one single-
// workgroup launch (per thread a contiguous run of edges: sum, block scan, write), and the
// transposed lists are written directly in order instead of by atomics plus a segment sort.
constexpr int kScan1Threads = 1024;
constexpr int64_t kScan1Max = 32768;  // one-workgroup scan up to this many counts (staged in LDS)

// count[i] = deg(atom[i]) - 1 for the multi-workgroup scan of larger graphs
__global__ void degree_count(const int32_t* __restrict__ atom, const int32_t* __restrict__ atom_rowptr, int64_t n,
                             int32_t* __restrict__ count) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int a = atom[i];
  const int c = atom_rowptr[a + 1] - atom_rowptr[a] - 1;
  count[i] = c > 0 ? c : 0;
}

// Exclusive scan of n <= kScan1Max counts deg(atom[i]) - 1 in ONE workgroup: the counts' gathers
// (atom[i], then atom_rowptr[a], atom_rowptr[a + 1]) kDegUnroll per thread at a time, every load of
// a batch in flight together, into LDS; each thread then scans a contiguous run; out[n] = total.
// One launch instead of a count launch + the three-phase scan for a training batch's line graph
// (round 3: the counts were a separate grid launch before this one-workgroup scan).
constexpr int kDegUnroll = 8;
__device__ __forceinline__ void src_rowptr_sym_body(const int32_t* __restrict__ edge_src,
                                                    const int32_t* __restrict__ atom_rowptr, int64_t E,
                                                    int32_t* __restrict__ src_rowptr, int* lds);
// sym_src (or NULL): also the symmetric graph's src_rowptr from edge_src = sym_src (src_rowptr_sym_body)
__global__ void __launch_bounds__(kScan1Threads) degree_scan_1wg(const int32_t* __restrict__ atom,
                                                                const int32_t* __restrict__ atom_rowptr, int64_t n,
                                                                int32_t* __restrict__ out,
                                                                const int32_t* __restrict__ sym_src = nullptr,
                                                                int32_t* __restrict__ src_rowptr = nullptr) {
  __shared__ int cnt[kScan1Max];
  __shared__ int lds[kScan1Threads / 64];
  const int tid = threadIdx.x;
  for (int64_t i0 = tid; i0 < n; i0 += static_cast<int64_t>(kScan1Threads) * kDegUnroll) {
    int a[kDegUnroll], d0[kDegUnroll], d1[kDegUnroll];
#pragma unroll
    for (int u = 0; u < kDegUnroll; ++u) {
      const int64_t i = i0 + static_cast<int64_t>(u) * kScan1Threads;
      a[u] = atom[i < n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < kDegUnroll; ++u) {
      d0[u] = atom_rowptr[a[u]];
      d1[u] = atom_rowptr[a[u] + 1];
    }
#pragma unroll
    for (int u = 0; u < kDegUnroll; ++u) {
      const int64_t i = i0 + static_cast<int64_t>(u) * kScan1Threads;
      const int c = d1[u] - d0[u] - 1;
      if (i < n) cnt[i] = c > 0 ? c : 0;
    }
  }
  __syncthreads();
  const int64_t per = (n + kScan1Threads - 1) / kScan1Threads;
  const int64_t lo = per * tid, hi = lo + per < n ? lo + per : n;
  int sum = 0;
  for (int64_t i = lo; i < hi; ++i) sum += cnt[i];
  int total;
  int run = block_exclusive_scan(sum, lds, &total);
  for (int64_t i = lo; i < hi; ++i) {
    const int c = cnt[i];
    cnt[i] = run;
    run += c;
  }
  __syncthreads();
  for (int64_t i = tid; i < n; i += kScan1Threads) out[i] = cnt[i];  // coalesced stores
  if (tid == 0) out[n] = total;
  if (src_rowptr) src_rowptr_sym_body(sym_src, atom_rowptr, n, src_rowptr, lds);  // (uniform)
}

// src_rowptr of a SYMMETRIC edge set from the atoms instead of the edges: source s = (b->k) has
// deg(b) - 1 triplets and b's out-edges are contiguous (edges sorted by source), so
//     src_rowptr[atom_rowptr[b] + j] = P[b] + j (deg(b) - 1),   P[b] = sum_{b' < b} deg(b') (deg(b') - 1),
// one scan over the atoms (contiguous atom_rowptr loads) instead of over the edges with two dependent
// gathers per edge (degree_scan_1wg: 12 us at config 2, this 3-4 us).  The atoms that own edges are
// 0 .. edge_src[E-1]; thread t takes a contiguous range of them.
__device__ __forceinline__ void src_rowptr_sym_body(const int32_t* __restrict__ edge_src,
                                                    const int32_t* __restrict__ atom_rowptr, int64_t E,
                                                    int32_t* __restrict__ src_rowptr, int* lds) {
  const int tid = threadIdx.x;
  const int64_t n = static_cast<int64_t>(edge_src[E - 1]) + 1;  // atoms 0 .. n-1 (the last owns edge E-1)
  const int64_t per = (n + kScan1Threads - 1) / kScan1Threads;
  const int64_t lo = per * tid < n ? per * tid : n, hi = lo + per < n ? lo + per : n;
  int sum = 0;
  for (int64_t b = lo; b < hi; ++b) {
    const int d = atom_rowptr[b + 1] - atom_rowptr[b];
    sum += d * (d > 0 ? d - 1 : 0);
  }
  int total;
  int run = block_exclusive_scan(sum, lds, &total);
  for (int64_t b = lo; b < hi; ++b) {
    const int r0 = atom_rowptr[b], d = atom_rowptr[b + 1] - r0, c = d > 0 ? d - 1 : 0;
    for (int j = 0; j < d; ++j) src_rowptr[r0 + j] = run + j * c;
    run += d * c;
  }
  if (tid == 0) src_rowptr[E] = total;
}

__global__ void __launch_bounds__(kScan1Threads) src_rowptr_sym_1wg(const int32_t* __restrict__ edge_src,
                                                                   const int32_t* __restrict__ atom_rowptr, int64_t E,
                                                                   int32_t* __restrict__ src_rowptr) {
  __shared__ int lds[kScan1Threads / 64];
  src_rowptr_sym_body(edge_src, atom_rowptr, E, src_rowptr, lds);
}

// out = exclusive scan of deg(atom[i]) - 1: one workgroup when it fits (counts and scan), else the
// counts by a grid of threads and the multi-workgroup scan
int degree_scan(const int32_t* atom, const int32_t* atom_rowptr, int64_t n, int32_t* out, int32_t* count,
                int32_t* partial, hipStream_t st) {
  if (n > 0 && n <= kScan1Max) {
    degree_scan_1wg<<<1, kScan1Threads, 0, st>>>(atom, atom_rowptr, n, out);
    return last_launch_status();
  }
  if (n > 0) {
    degree_count<<<blocks_for(n, 256), 256, 0, st>>>(atom, atom_rowptr, n, count);
    if (int rc = last_launch_status()) return rc;
  }
  return exclusive_scan(count, n, out, partial, st);
}

// Source s = (b->k) lists its triplets (s -> e), e = (a->b) over b's neighbours a != k in
// ascending a (= ascending edge id of e = ascending triplet id).  In e's destination list (b's
// out-edges minus b->a, ascending) s sits at rank_b(k) - [rank_b(a) < rank_b(k)], so the triplet
// id is trip_rowptr[e] plus that; e itself is found in a's sorted out-list.  A group of 8 lanes per
// source walks b's neighbours 8 at a time (one search each, in parallel) and compacts with a
// ballot, as the triplet emitter does.
__device__ __forceinline__ void transpose_group(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                                const int32_t* __restrict__ atom_rowptr,
                                                const int32_t* __restrict__ trip_rowptr,
                                                const int32_t* __restrict__ src_rowptr, int64_t E,
                                                int32_t* __restrict__ src_perm, int32_t* __restrict__ src_dst) {
  const int64_t gtid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t s = gtid / kEmitGroup;
  const int sub = threadIdx.x & (kEmitGroup - 1);
  const int lane = threadIdx.x & 63;
  const uint64_t group_mask = ((1ull << kEmitGroup) - 1) << (lane & ~(kEmitGroup - 1));
  const bool valid = s < E;
  int b = 0, k = 0, lo = 0, hi = 0, p = 0;
  if (valid) {
    b = src[s];
    k = dst[s];
    lo = atom_rowptr[b];
    hi = atom_rowptr[b + 1];
    p = src_rowptr[s];
  }
  const int rank_k = static_cast<int>(s) - lo;
  for (int base = lo; __any(valid && base < hi); base += kEmitGroup) {
    const int idx = base + sub;
    const bool in = valid && idx < hi;
    const int a = in ? dst[idx] : 0;
    const bool keep = in && a != k;
    int tid_out = 0, e = 0;
    if (keep) {
      e = lower_bound(dst, atom_rowptr[a], atom_rowptr[a + 1], b);  // edge a->b (symmetric graph)
      tid_out = trip_rowptr[e] + rank_k - (idx - lo < rank_k ? 1 : 0);
    }
    const uint64_t ball = __ballot(keep) & group_mask;
    const int q = p + __popcll(ball & ((1ull << lane) - 1));
    if (keep) {
      src_perm[q] = tid_out;
      if (src_dst) src_dst[q] = e;
    }
    p += __popcll(ball);
  }
}

__global__ void transpose_sym_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                     const int32_t* __restrict__ atom_rowptr, const int32_t* __restrict__ trip_rowptr,
                                     const int32_t* __restrict__ src_rowptr, int64_t E,
                                     int32_t* __restrict__ src_perm, int32_t* __restrict__ src_dst) {
  transpose_group(src, dst, atom_rowptr, trip_rowptr, src_rowptr, E, src_perm, src_dst);
}

// both per-edge passes of a symmetric line graph in one grid: edge g emits its triplets as a
// destination (emit_group) and lists them as a source (transpose_group, which reads only trip_rowptr)
__global__ void emit_transpose_sym_kernel(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                          const int32_t* __restrict__ atom_rowptr,
                                          const int32_t* __restrict__ trip_rowptr,
                                          const int32_t* __restrict__ src_rowptr, int64_t E, int64_t T,
                                          int32_t* __restrict__ trip_src, int32_t* __restrict__ trip_dst,
                                          int32_t* __restrict__ atom_j, int32_t* __restrict__ atom_i,
                                          int32_t* __restrict__ atom_k, int32_t* __restrict__ src_perm,
                                          int32_t* __restrict__ src_dst, int32_t* __restrict__ edge_rev,
                                          int32_t* __restrict__ rev_trip) {
  emit_group(src, dst, atom_rowptr, trip_rowptr, E, T, trip_src, trip_dst, atom_j, atom_i, atom_k, edge_rev, rev_trip);
  transpose_group(src, dst, atom_rowptr, trip_rowptr, src_rowptr, E, src_perm, src_dst);
}

// ----------------------------------------------------------------------------- per-molecule row pointers
// The row pointers of a SYMMETRIC line graph of a batch of molecules (every edge joins two atoms of one
// molecule: a PyG batch), one workgroup per molecule m, nothing shared between workgroups: its atoms
// a0 .. a1 - 1 (mol_ptr) own its edges E0 .. E1 - 1 (line_ptr), so
//   atom_rowptr[b] = E0 + #{e in molecule : src e < b}       (a histogram of the molecule's sources in LDS),
//   trip_rowptr[e] = T0 + sum_{e' in [E0, e)} (deg(dst e') - 1),   T0 = sum_{m' < m} mol_trips[m'],
// the degrees read from the same LDS histogram and T0 from the host's (or x2g_batch_meta's) per-molecule
// triplet counts.  Replaces the row-pointer grid and the one-workgroup scan over all E edges (24.6 us at
// config 2 on one CU) with one launch of B short workgroups.
constexpr int kMolThreads = 256;

__global__ void __launch_bounds__(kMolThreads) mol_rowptr_sym_kernel(
    const int32_t* __restrict__ edge_src, const int32_t* __restrict__ edge_dst, const int32_t* __restrict__ mol_ptr,
    const int32_t* __restrict__ line_ptr, const int64_t* __restrict__ mol_trips, int64_t B, int64_t E, int64_t N,
    int64_t T, int32_t* __restrict__ atom_rowptr, int32_t* __restrict__ trip_rowptr) {
  extern __shared__ int deg[];  // [a1 - a0]
  __shared__ int lds[kMolThreads / 64];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int a0 = mol_ptr[m], a1 = mol_ptr[m + 1], e0 = line_ptr[m], e1 = line_ptr[m + 1];
  const int na = a1 - a0;
  for (int i = tid; i < na; i += kMolThreads) deg[i] = 0;
  // T0: the triplets of the molecules before this one
  int64_t part = 0;
  for (int64_t i = tid; i < m; i += kMolThreads) part += mol_trips[i];
  int t0;
  block_exclusive_scan(static_cast<int>(part), lds, &t0);  // (its barriers also order the zeroing)
  for (int e = e0 + tid; e < e1; e += kMolThreads) {
    const int b = edge_src[e] - a0;
    if (b >= 0 && b < na) atomicAdd(&deg[b], 1);  // (a molecule's edges join its own atoms: host contract)
  }
  __syncthreads();
  // atom_rowptr over the molecule's atoms, chunk by chunk with a carry
  int carry = e0;
  for (int c = 0; c < na; c += kMolThreads) {
    const int i = c + tid;
    const int d = i < na ? deg[i] : 0;
    int tot;
    const int pre = block_exclusive_scan(d, lds, &tot);
    if (i < na) atom_rowptr[a0 + i] = carry + pre;
    carry += tot;
  }
  // trip_rowptr over the molecule's edges
  carry = t0;
  for (int c = e0; c < e1; c += kMolThreads) {
    const int e = c + tid;
    int cnt = 0;
    if (e < e1) {
      const int b = edge_dst[e] - a0;
      cnt = (b >= 0 && b < na) ? deg[b] - 1 : 0;
      cnt = cnt > 0 ? cnt : 0;
    }
    int tot;
    const int pre = block_exclusive_scan(cnt, lds, &tot);
    if (e < e1) trip_rowptr[e] = carry + pre;
    carry += tot;
  }
  if (m == B - 1 && tid == 0) {
    atom_rowptr[N] = static_cast<int32_t>(E);
    trip_rowptr[E] = static_cast<int32_t>(T);
  }
}

// ----------------------------------------------------------------------------- batch metadata
// A PyG-style batch made elsewhere (the drop-in's real caller, trainer.py:37-40: a DataLoader Batch of
// xgnn.py:41-52's keys) carries neither per-molecule triplet counts nor x2gnn's int32 index forms.  Both
// come from the device in one pass: per atom its element and the molecules' atom row pointer (CSR of
// batch[], the rowptr_kernel rule); per edge e = (a->b) the int32 endpoints, their elements and the
// molecules' edge row pointer (CSR of batch[src[]]); then per edge its triplet count deg(b) - [b->a
// exists] (the reverse found by binary search in b's sorted out-list) summed into its molecule batch[a]
// (integer atomics: exact, order-independent).  Everything the host needs lands in one int64 block
// info = [mol_ptr (B+1) | line_ptr (B+1) | triplets (B) | flags (4)], read back with one copy; flags:
// [0] edges without a reverse (0 = symmetric), [1] the largest out-degree, [2] edges out of (src, dst)
// order, repeated or out of range (the builders need a sorted simple edge list), [3] edges joining two
// molecules (0: the per-molecule builder x2g_vertex_to_edge_sym_mol applies).
__device__ __forceinline__ void ptr_fill(int64_t prev, int64_t cur, int64_t n_seg, int32_t val,
                                         int32_t* __restrict__ rowptr, int64_t* __restrict__ rowptr64) {
  if (prev < -1) prev = -1;
  if (cur > n_seg) cur = n_seg;
  for (int64_t s = prev + 1; s <= cur; ++s) {
    rowptr[s] = val;
    rowptr64[s] = val;
  }
}

// (launched first: also zeroes the triplet counts and flags the later kernels add into)
__global__ void batch_meta_atoms(const int64_t* __restrict__ x, const int64_t* __restrict__ batch, int64_t N,
                                 int64_t B, int32_t* __restrict__ atom_type, int32_t* __restrict__ mol_ptr,
                                 int64_t* __restrict__ info) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < B + 4) info[2 * (B + 1) + i] = 0;
  if (i > N) return;
  auto mol_of = [&](int64_t a) -> int64_t { return batch ? batch[a] : 0; };
  if (i == N) {
    ptr_fill(N > 0 ? mol_of(N - 1) : -1, B, B, static_cast<int32_t>(N), mol_ptr, info);
    return;
  }
  atom_type[i] = static_cast<int32_t>(x[i]);
  ptr_fill(i > 0 ? mol_of(i - 1) : -1, mol_of(i), B, static_cast<int32_t>(i), mol_ptr, info);
}

__global__ void batch_meta_edges(const int64_t* __restrict__ ei, const int64_t* __restrict__ x,
                                 const int64_t* __restrict__ batch, int64_t E, int64_t N, int64_t B,
                                 int32_t* __restrict__ src, int32_t* __restrict__ dst, int32_t* __restrict__ src_type,
                                 int32_t* __restrict__ dst_type, int32_t* __restrict__ line_ptr,
                                 int32_t* __restrict__ atom_rowptr, int64_t* __restrict__ info) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e > E) return;
  unsigned long long* flags = reinterpret_cast<unsigned long long*>(info + 3 * B + 2);
  int64_t* lp64 = info + (B + 1);
  auto mol_of = [&](int64_t a) -> int64_t { return (batch && a >= 0 && a < N) ? batch[a] : 0; };
  // the source-atom row pointer of the edges (rowptr_kernel's rule over src, clamped to [0, N])
  {
    const int64_t prev = e > 0 ? ei[e - 1] : -1, cur = e < E ? ei[e] : N;
    for (int64_t s = (prev < -1 ? -1 : prev) + 1; s <= (cur > N ? N : cur); ++s) atom_rowptr[s] = static_cast<int32_t>(e);
  }
  if (e == E) {  // the edge row pointer's tail
    ptr_fill(E > 0 ? mol_of(ei[E - 1]) : -1, B, B, static_cast<int32_t>(E), line_ptr, lp64);
    return;
  }
  const int64_t a = ei[e], b = ei[E + e];
  src[e] = static_cast<int32_t>(a);
  dst[e] = static_cast<int32_t>(b);
  const bool ok = a >= 0 && a < N && b >= 0 && b < N;
  src_type[e] = ok ? static_cast<int32_t>(x[a]) : 0;
  dst_type[e] = ok ? static_cast<int32_t>(x[b]) : 0;
  if (!ok) atomicAdd(&flags[2], 1ull);
  if (ok && mol_of(a) != mol_of(b)) atomicAdd(&flags[3], 1ull);  // an edge between two molecules
  if (e > 0) {
    const int64_t pa = ei[e - 1], pb = ei[E + e - 1];
    if (pa > a || (pa == a && pb >= b)) atomicAdd(&flags[2], 1ull);
  }
  ptr_fill(e > 0 ? mol_of(ei[e - 1]) : -1, mol_of(a), B, static_cast<int32_t>(e), line_ptr, lp64);
}

__global__ void batch_meta_count(const int32_t* __restrict__ src, const int32_t* __restrict__ dst,
                                 const int32_t* __restrict__ atom_rowptr, const int64_t* __restrict__ batch,
                                 int64_t E, int64_t N, int64_t B, int64_t* __restrict__ info) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= E) return;
  unsigned long long* trips = reinterpret_cast<unsigned long long*>(info + 2 * (B + 1));
  unsigned long long* flags = trips + B;
  const int a = src[e], b = dst[e];
  if (a < 0 || a >= N || b < 0 || b >= N) return;  // (flagged by batch_meta_edges)
  const int lo = atom_rowptr[b], hi = atom_rowptr[b + 1];
  const int p = lower_bound(dst, lo, hi, a);
  const int has_rev = (p < hi && dst[p] == a) ? 1 : 0;
  if (!has_rev) atomicAdd(&flags[0], 1ull);
  if (e == atom_rowptr[a]) atomicMax(&flags[1], static_cast<unsigned long long>(atom_rowptr[a + 1] - atom_rowptr[a]));
  const int64_t m = batch ? batch[a] : 0;
  if (m >= 0 && m < B) atomicAdd(&trips[m], static_cast<unsigned long long>(hi - lo - has_rev));
}

}  // namespace x2g

using namespace x2g;

X2G_API int x2g_batch_meta(const int64_t* edge_index, const int64_t* x, const int64_t* batch, int64_t num_edges,
                           int64_t num_nodes, int64_t num_graphs, int32_t* edge_src, int32_t* edge_dst,
                           int32_t* src_type, int32_t* dst_type, int32_t* atom_type, int32_t* line_ptr,
                           int32_t* mol_ptr, int32_t* atom_rowptr, int64_t* info, void* stream) {
  if (num_edges < 0 || num_nodes < 0 || num_graphs < 0 || !atom_rowptr || !info || !line_ptr || !mol_ptr ||
      (num_nodes > 0 && (!x || !atom_type)))
    return X2G_EINVAL;
  if (num_edges > 0 && (!edge_index || !edge_src || !edge_dst || !src_type || !dst_type)) return X2G_EINVAL;
  if (num_edges > 0x7fffffff || num_nodes > 0x7fffffff) return X2G_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  // threads: N + 1 atom slots, and B + 4 to zero the triplet counts and the four flags
  const int64_t na = (num_nodes + 1 > num_graphs + 4 ? num_nodes + 1 : num_graphs + 4);
  batch_meta_atoms<<<blocks_for(na, 256), 256, 0, st>>>(x, batch, num_nodes, num_graphs, atom_type, mol_ptr, info);
  if (int rc = last_launch_status()) return rc;
  batch_meta_edges<<<blocks_for(num_edges + 1, 256), 256, 0, st>>>(edge_index, x, batch, num_edges, num_nodes,
                                                                   num_graphs, edge_src, edge_dst, src_type, dst_type,
                                                                   line_ptr, atom_rowptr, info);
  if (int rc = last_launch_status()) return rc;
  if (num_edges > 0)
    batch_meta_count<<<blocks_for(num_edges, 256), 256, 0, st>>>(edge_src, edge_dst, atom_rowptr, batch, num_edges,
                                                                 num_nodes, num_graphs, info);
  return last_launch_status();
}

X2G_API int x2g_abi_version(void) { return 17; }

X2G_API const char* x2g_status_string(int status) {
  switch (status) {
    case X2G_OK: return "ok";
    case X2G_EINVAL: return "X2G_EINVAL: bad size or null pointer";
    case X2G_EUNSUPPORTED: return "X2G_EUNSUPPORTED: shape outside the compiled kernel set";
    case X2G_EWORKSPACE: return "X2G_EWORKSPACE: workspace too small";
    default: return hipGetErrorString(static_cast<hipError_t>(status));
  }
}

X2G_API int x2g_csr_rowptr(const int32_t* keys, int64_t n, int64_t n_seg, int32_t* rowptr, void* stream) {
  if (n < 0 || n_seg < 0 || !rowptr || (n > 0 && !keys)) return X2G_EINVAL;
  rowptr_kernel<<<blocks_for(n + 1, 256), 256, 0, as_stream(stream)>>>(keys, n, n_seg, rowptr);
  return last_launch_status();
}

X2G_API int x2g_csr_rowptr_checked(const int32_t* keys, int64_t n, int64_t n_seg, int32_t* rowptr,
                                   int32_t* status, void* stream) {
  if (n < 0 || n_seg < 0 || !rowptr || !status || (n > 0 && !keys)) return X2G_EINVAL;
  if (n_seg + 1 > INT32_MAX || n > INT32_MAX) return X2G_EINVAL;
  hipStream_t st = as_stream(stream);
  const hipError_t me = hipMemsetAsync(status, 0, sizeof(int32_t), st);
  if (me != hipSuccess) return static_cast<int>(me);
  const int64_t m = n > n_seg + 1 ? n : n_seg + 1;
  rowptr_checked_kernel<<<blocks_for(m, 256), 256, 0, st>>>(keys, n, n_seg, rowptr, status);
  return last_launch_status();
}

X2G_API size_t x2g_vertex_to_edge_workspace(int64_t num_edges, int64_t num_nodes) {
  const int64_t n = num_edges > num_nodes ? num_edges : num_nodes;
  // counts/cursor [n] + scan partials, 256-byte aligned
  const int64_t ints = 2 * (n + 64) + scan_partials_ints(n + 1) + 64;
  return static_cast<size_t>(ints) * sizeof(int32_t);
}

X2G_API int x2g_vertex_to_edge(const int32_t* edge_src, const int32_t* edge_dst, int64_t E, int64_t N,
                               int64_t T, int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src,
                               int32_t* trip_dst, int32_t* atom_j, int32_t* atom_i, int32_t* atom_k,
                               void* workspace, size_t workspace_bytes, void* stream) {
  if (E < 0 || N < 0 || T < 0 || !atom_rowptr || !trip_rowptr) return X2G_EINVAL;
  if (E > 0 && (!edge_src || !edge_dst)) return X2G_EINVAL;
  if (T > 0 && (!trip_src || !trip_dst)) return X2G_EINVAL;
  if (workspace_bytes < x2g_vertex_to_edge_workspace(E, N) || !workspace) return X2G_EWORKSPACE;
  hipStream_t st = as_stream(stream);
  int32_t* count = static_cast<int32_t*>(workspace);
  const int64_t n = E > N ? E : N;
  int32_t* partial = count + 2 * (n + 64);
  int rc = x2g_csr_rowptr(edge_src, E, N, atom_rowptr, stream);
  if (rc) return rc;
  if (E > 0) {
    triplet_count_kernel<<<blocks_for(E, 256), 256, 0, st>>>(edge_src, edge_dst, atom_rowptr, E, count);
    if ((rc = last_launch_status())) return rc;
  }
  if ((rc = exclusive_scan(count, E, trip_rowptr, partial, st))) return rc;
  if (E > 0) {
    triplet_emit_kernel<<<blocks_for(E * kEmitGroup, 256), 256, 0, st>>>(
        edge_src, edge_dst, atom_rowptr, trip_rowptr, E, T, trip_src, trip_dst, atom_j, atom_i, atom_k, nullptr,
        nullptr);
  }
  return last_launch_status();
}

// src_dst[p] = trip_dst[src_perm[p]]: the destination of each source-major position
__global__ void gather_dst_kernel(const int32_t* __restrict__ perm, const int32_t* __restrict__ tdst, int64_t T,
                                  int32_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < T) out[i] = tdst[perm[i]];
}

X2G_API int x2g_line_graph_transpose(const int32_t* trip_src, const int32_t* trip_dst, int64_t T, int64_t E,
                                     int32_t* src_rowptr, int32_t* src_perm, int32_t* src_dst, void* workspace,
                                     size_t workspace_bytes, void* stream) {
  if (T < 0 || E < 0 || !src_rowptr || (T > 0 && (!trip_src || !src_perm))) return X2G_EINVAL;
  if (T > 0 && src_dst && !trip_dst) return X2G_EINVAL;
  if (workspace_bytes < x2g_vertex_to_edge_workspace(E, 0) || !workspace) return X2G_EWORKSPACE;
  hipStream_t st = as_stream(stream);
  int32_t* count = static_cast<int32_t*>(workspace);
  int32_t* cursor = count + (E + 64);
  int32_t* partial = count + 2 * (E + 64);
  int rc;
  const hipError_t me = hipMemsetAsync(count, 0, sizeof(int32_t) * (2 * (E + 64)), st);
  if (me != hipSuccess) return static_cast<int>(me);
  if (T > 0) {
    count_by_key<<<blocks_for(T, 256), 256, 0, st>>>(trip_src, T, count);
    if ((rc = last_launch_status())) return rc;
  }
  if ((rc = exclusive_scan(count, E, src_rowptr, partial, st))) return rc;
  if (T > 0) {
    fill_by_key<<<blocks_for(T, 256), 256, 0, st>>>(trip_src, T, src_rowptr, cursor, src_perm);
    sort_segments<<<blocks_for(E, 256), 256, 0, st>>>(src_rowptr, E, src_perm);
    if (src_dst) gather_dst_kernel<<<blocks_for(T, 256), 256, 0, st>>>(src_perm, trip_dst, T, src_dst);
  }
  return last_launch_status();
}

X2G_API int x2g_vertex_to_edge_sym(const int32_t* edge_src, const int32_t* edge_dst, int64_t E, int64_t N, int64_t T,
                                   int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src, int32_t* trip_dst,
                                   int32_t* atom_j, int32_t* atom_i, int32_t* atom_k, int32_t* edge_rev,
                                   int32_t* rev_trip, void* workspace, size_t workspace_bytes, void* stream) {
  if (E < 0 || N < 0 || T < 0 || !atom_rowptr || !trip_rowptr) return X2G_EINVAL;
  if (!edge_rev != !rev_trip) return X2G_EINVAL;
  if (E > 0 && (!edge_src || !edge_dst)) return X2G_EINVAL;
  if (T > 0 && (!trip_src || !trip_dst)) return X2G_EINVAL;
  if (workspace_bytes < x2g_vertex_to_edge_workspace(E, N) || !workspace) return X2G_EWORKSPACE;
  hipStream_t st = as_stream(stream);
  int32_t* count = static_cast<int32_t*>(workspace);
  const int64_t n = E > N ? E : N;
  int32_t* partial = count + 2 * (n + 64);
  int rc = x2g_csr_rowptr(edge_src, E, N, atom_rowptr, stream);
  if (rc) return rc;
  if ((rc = degree_scan(edge_dst, atom_rowptr, E, trip_rowptr, count, partial, st))) return rc;
  if (E > 0) {
    triplet_emit_kernel<<<blocks_for(E * kEmitGroup, 256), 256, 0, st>>>(
        edge_src, edge_dst, atom_rowptr, trip_rowptr, E, T, trip_src, trip_dst, atom_j, atom_i, atom_k, edge_rev,
        rev_trip);
  }
  return last_launch_status();
}

X2G_API int x2g_vertex_to_edge_sym_mol(const int32_t* edge_src, const int32_t* edge_dst, int64_t E, int64_t N,
                                       int64_t T, const int32_t* mol_ptr, const int32_t* line_ptr,
                                       const int64_t* mol_trips, int64_t num_mols, int32_t max_mol_atoms,
                                       int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src,
                                       int32_t* trip_dst, int32_t* atom_j, int32_t* atom_i, int32_t* atom_k,
                                       int32_t* edge_rev, int32_t* rev_trip, void* stream) {
  if (E < 0 || N < 0 || T < 0 || num_mols <= 0 || max_mol_atoms < 0 || !atom_rowptr || !trip_rowptr || !mol_ptr ||
      !line_ptr || !mol_trips)
    return X2G_EINVAL;
  if (!edge_rev != !rev_trip) return X2G_EINVAL;
  if (E > 0 && (!edge_src || !edge_dst)) return X2G_EINVAL;
  if (T > 0 && (!trip_src || !trip_dst)) return X2G_EINVAL;
  if (T >= (int64_t(1) << 31) || E >= (int64_t(1) << 31) || num_mols >= (int64_t(1) << 31) ||
      static_cast<size_t>(max_mol_atoms) * 4 > 64 * 1024)
    return X2G_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  mol_rowptr_sym_kernel<<<static_cast<unsigned>(num_mols), kMolThreads, static_cast<size_t>(max_mol_atoms) * 4, st>>>(
      edge_src, edge_dst, mol_ptr, line_ptr, mol_trips, num_mols, E, N, T, atom_rowptr, trip_rowptr);
  if (int rc = last_launch_status()) return rc;
  if (E > 0) {
    triplet_emit_kernel<<<blocks_for(E * kEmitGroup, 256), 256, 0, st>>>(
        edge_src, edge_dst, atom_rowptr, trip_rowptr, E, T, trip_src, trip_dst, atom_j, atom_i, atom_k, edge_rev,
        rev_trip);
  }
  return last_launch_status();
}

X2G_API int x2g_line_graph_transpose_sym(const int32_t* edge_src, const int32_t* edge_dst, const int32_t* atom_rowptr,
                                         const int32_t* trip_rowptr, int64_t E, int32_t* src_rowptr,
                                         int32_t* src_perm, int32_t* src_dst, void* workspace, size_t workspace_bytes,
                                         void* stream) {
  if (E < 0 || !src_rowptr || (E > 0 && (!edge_src || !edge_dst || !atom_rowptr || !trip_rowptr || !src_perm)))
    return X2G_EINVAL;
  if (workspace_bytes < x2g_vertex_to_edge_workspace(E, 0) || !workspace) return X2G_EWORKSPACE;
  hipStream_t st = as_stream(stream);
  int32_t* count = static_cast<int32_t*>(workspace);
  int32_t* partial = count + 2 * (E + 64);
  int rc;
  if (E > 0) {
    src_rowptr_sym_1wg<<<1, kScan1Threads, 0, st>>>(edge_src, atom_rowptr, E, src_rowptr);
    if ((rc = last_launch_status())) return rc;
  } else if ((rc = degree_scan(edge_src, atom_rowptr, E, src_rowptr, count, partial, st))) {
    return rc;
  }
  if (E > 0)
    transpose_sym_kernel<<<blocks_for(E * kEmitGroup, 256), 256, 0, st>>>(edge_src, edge_dst, atom_rowptr, trip_rowptr,
                                                                          src_rowptr, E, src_perm, src_dst);
  return last_launch_status();
}

X2G_API int x2g_line_graph_sym_build(const int32_t* edge_src, const int32_t* edge_dst, int64_t E, int64_t N,
                                     int64_t T, int32_t* atom_rowptr, int32_t* trip_rowptr, int32_t* trip_src,
                                     int32_t* trip_dst, int32_t* atom_j, int32_t* atom_i, int32_t* atom_k,
                                     int32_t* src_rowptr, int32_t* src_perm, int32_t* src_dst, int32_t* edge_rev,
                                     int32_t* rev_trip, void* workspace, size_t workspace_bytes, void* stream) {
  if (E < 0 || N < 0 || T < 0 || !atom_rowptr || !trip_rowptr || !src_rowptr) return X2G_EINVAL;
  if (!edge_rev != !rev_trip) return X2G_EINVAL;
  if (E > 0 && (!edge_src || !edge_dst)) return X2G_EINVAL;
  if (T > 0 && (!trip_src || !trip_dst || !src_perm)) return X2G_EINVAL;
  if (workspace_bytes < x2g_vertex_to_edge_workspace(E, N) || !workspace) return X2G_EWORKSPACE;
  if (E == 0 || E > kScan1Max) {  // outside the one-workgroup scan: the two entry points in turn
    if (int rc = x2g_vertex_to_edge_sym(edge_src, edge_dst, E, N, T, atom_rowptr, trip_rowptr, trip_src, trip_dst,
                                        atom_j, atom_i, atom_k, edge_rev, rev_trip, workspace, workspace_bytes,
                                        stream))
      return rc;
    return x2g_line_graph_transpose_sym(edge_src, edge_dst, atom_rowptr, trip_rowptr, E, src_rowptr, src_perm,
                                        src_dst, workspace, workspace_bytes, stream);
  }
  hipStream_t st = as_stream(stream);
  int rc = x2g_csr_rowptr(edge_src, E, N, atom_rowptr, stream);
  if (rc) return rc;
  degree_scan_1wg<<<1, kScan1Threads, 0, st>>>(edge_dst, atom_rowptr, E, trip_rowptr, edge_src, src_rowptr);
  if ((rc = last_launch_status())) return rc;
  emit_transpose_sym_kernel<<<blocks_for(E * kEmitGroup, 256), 256, 0, st>>>(
      edge_src, edge_dst, atom_rowptr, trip_rowptr, src_rowptr, E, T, trip_src, trip_dst, atom_j, atom_i, atom_k,
      src_perm, src_dst, edge_rev, rev_trip);
  return last_launch_status();
}

namespace x2g {

// ----------------------------------------------------------------------------- center-atom schedule
// The center-atom attention kernels' workgroup schedule made on the device (a batch made elsewhere — the
// reference trainer's PyG DataLoader batch, trainer.py:25-27,37-40 — carries none; x2gnn's collate makes the
// same kind of schedule on the host, data.center_packs):
//   * the fused forward's UNITS: per window of 64 consecutive atoms, its atoms by decreasing degree packed
//     best-fit into units of <= 16 rows and <= 16 members (an atom of degree >= 16 alone, atoms without edges
//     16 to a unit), one wave per window: the units' remaining rows sit one per lane and each atom's best
//     fit is a 4-step ballot minimum over the lanes (no cross-lane shuffles in the serial loop).  A unit may
//     span molecules (nothing in the center kernels is per molecule).
//   * the units then in ONE list by decreasing largest degree (collate's order: the longest workgroups start
//     first, so no heavy unit is dispatched at the launch's tail) and compact (units 0 .. U - 1, slots U .. N
//     empty): a histogram of the units' keys and member counts, its suffix sums, and each unit's place from
//     one 64-bit atomic per unit on its key's (units, members) cursor — the unit index and the first member
//     position come from the same atomic, so pack_ptr stays monotonic.
//   * atom_info per position of pack_order: (atom, first out-edge, degree, src_row of its first out-edge).
//   * center_order: every atom by decreasing degree (the backward's one-atom workgroups, longest first): the
//     degree histogram's suffix sums and a per-degree cursor.
// The order among atoms (units) of one degree (key) follows the atomics: no output of the center kernels
// depends on it (each atom's block is computed whole by one workgroup in a fixed order).
// Round 6's first forms, units in per-molecule (then per-window) slot order with empty slots between them,
// ran the fused forwards 45 % (config 2) and 50 % (config 5) slower than collate's ordered list
// (profiles/r6j_sched_kernels.txt): heavy units dispatched late and empty workgroups interleaved.
constexpr int kSchedCap = 16;       // rows per unit (data.CENTER_PACK_ROWS)
constexpr int kSchedMembers = 16;   // atoms per unit (data.CENTER_PACK_MEMBERS)
constexpr int kSchedDeg = 128;      // degree / key bins (X2G_CENTER_MAX_DEGREE; larger degrees share the last)
constexpr int kSchedWin = 64;       // atoms per window (one wave)
constexpr int kSchedBins = kSchedDeg + 1;

// workspace (int32 words): atom degree histogram and cursors, unit (units << 32 | members) histogram and
// cursors (64-bit), the three suffix sums, then per atom slot the window-local pack order, the unit word of
// the window's unit slots and per window-local position (unit, index in it)
struct SchedWs {
  int32_t* hist;
  int32_t* acur;
  unsigned long long* ubin;
  unsigned long long* ucur;
  int32_t* apre;
  int32_t* upre;
  int32_t* mpre;
  int32_t* t_order;
  int32_t* t_unit;
  int32_t* t_posu;
};
constexpr int kSchedUbinWord = (2 * kSchedBins + 1) & ~1;           // 8-byte aligned
constexpr int kSchedApreWord = kSchedUbinWord + 4 * kSchedBins;      // (the memset clears the words before)
constexpr int kSchedTempWord = kSchedApreWord + 3 * kSchedBins;

inline SchedWs sched_ws(void* base, int64_t N) {
  int32_t* w = static_cast<int32_t*>(base);
  SchedWs r;
  r.hist = w;
  r.acur = w + kSchedBins;
  r.ubin = reinterpret_cast<unsigned long long*>(w + kSchedUbinWord);
  r.ucur = r.ubin + kSchedBins;
  r.apre = w + kSchedApreWord;
  r.upre = r.apre + kSchedBins;
  r.mpre = r.upre + kSchedBins;
  r.t_order = w + kSchedTempWord;
  r.t_unit = r.t_order + N;
  r.t_posu = r.t_unit + N;
  return r;
}

// minimum over the wave's lanes of a 4-bit value v among the lanes with ok set: the mask of the lanes
// holding it (0 when no lane is ok), by ballots from the top bit down
__device__ __forceinline__ unsigned long long ballot_min4(bool ok, int v) {
  unsigned long long cand = __ballot(ok);
#pragma unroll
  for (int bit = 3; bit >= 0; --bit) {
    const unsigned long long zero = cand & __ballot(((v >> bit) & 1) == 0);
    if (zero) cand = zero;
  }
  return cand;
}

__global__ void __launch_bounds__(64) center_pack_window_kernel(const int32_t* __restrict__ rowptr, int64_t N,
                                                                SchedWs ws) {
  __shared__ int sd[kSchedWin], sa[kSchedWin];
  const int lane = threadIdx.x;
  const int a0 = kSchedWin * static_cast<int>(blockIdx.x);
  const int na = static_cast<int>(N - a0 < kSchedWin ? N - a0 : kSchedWin);
  const int d = lane < na ? rowptr[a0 + lane + 1] - rowptr[a0 + lane] : -1;
  if (lane < na) atomicAdd(&ws.hist[min(d, kSchedDeg)], 1);
  int rank = 0;  // by decreasing degree, ties by index
  for (int k = 0; k < na; ++k) {
    const int dk = __builtin_amdgcn_readlane(d, k);
    rank += (dk > d || (dk == d && k < lane)) ? 1 : 0;
  }
  if (lane < na) {
    sd[rank] = d;
    sa[rank] = lane;
  }
  __syncthreads();
  const int sdv = lane < na ? sd[lane] : 0;  // lane r: the r-th degree (read below with readlane: no LDS
                                             // round trip in the serial loop)
  // unit u's state in lane u: rows left, members, whether it holds atoms without edges, its key (the degree
  // of its first, largest atom); atom r's unit and index in it end in lane r
  int space = 0, mem = 0, zero = 0, key = 0, nu = 0, my_u = 0, my_idx = 0;
  for (int r = 0; r < na; ++r) {
    const int dr = __builtin_amdgcn_readlane(sdv, r);
    const bool open = lane < nu && mem < kSchedMembers;
    unsigned long long m = 0;
    if (dr > 0 && dr < kSchedCap)  // best fit: the fullest unit that takes it (lowest lane on ties)
      m = ballot_min4(open && !zero && space >= dr, space);
    else if (dr == 0)  // atoms without edges: with each other
      m = __ballot(open && zero);
    int u;
    if (m == 0) {
      u = nu++;
      if (lane == u) {
        space = dr >= kSchedCap ? 0 : kSchedCap - dr;
        zero = dr == 0;
        key = min(dr, kSchedDeg);
      }
    } else {
      u = static_cast<int>(__builtin_ctzll(m));
      if (lane == u) space -= dr;
    }
    const int before = __builtin_amdgcn_readlane(mem, u);
    if (lane == u) ++mem;
    if (lane == r) {
      my_u = u;
      my_idx = before;
    }
  }
  // the units' window-local first positions: exclusive scan of their member counts
  int inc = lane < nu ? mem : 0;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  const int start = inc - (lane < nu ? mem : 0);
  const int ustart = __shfl(start, my_u, 64);
  if (lane < na) {
    ws.t_order[a0 + ustart + my_idx] = a0 + sa[lane];
    ws.t_posu[a0 + ustart + my_idx] = (my_u << 8) | my_idx;
  }
  if (lane < na) {
    if (lane < nu) {
      ws.t_unit[a0 + lane] = (key << 16) | (start << 8) | mem;
      atomicAdd(&ws.ubin[key], (1ull << 32) | static_cast<unsigned long long>(mem));
    } else {
      ws.t_unit[a0 + lane] = -1;
    }
  }
}

// suffix sums over the bins (largest key first) and the empty slots' pack_ptr
__global__ void __launch_bounds__(256) center_sched_scan_kernel(int64_t N, SchedWs ws, int32_t* __restrict__ pack_ptr) {
  __shared__ int h[kSchedBins], uu[kSchedBins], mm[kSchedBins];
  __shared__ int total_units;
  const int t = threadIdx.x;
  if (t < kSchedBins) {
    h[t] = ws.hist[t];
    const unsigned long long b = ws.ubin[t];
    uu[t] = static_cast<int>(b >> 32);
    mm[t] = static_cast<int>(b & 0xffffffffull);
  }
  __syncthreads();
  if (t < kSchedBins) {
    int sa = 0, su = 0, sm = 0;
    for (int e = kSchedDeg; e > t; --e) {
      sa += h[e];
      su += uu[e];
      sm += mm[e];
    }
    ws.apre[t] = sa;
    ws.upre[t] = su;
    ws.mpre[t] = sm;
    if (t == 0) total_units = su + uu[0];
  }
  __syncthreads();
  for (int64_t s = total_units + t; s <= N; s += 256) pack_ptr[s] = static_cast<int32_t>(N);
}

// one wave per window: its units' places (one atomic per unit), then its atoms' positions (lane p: the
// window's p-th atom in pack order) — every dependent chain a few loads long
__global__ void __launch_bounds__(64) center_sched_place_kernel(const int32_t* __restrict__ rowptr,
                                                                const int32_t* __restrict__ src_row, int64_t N,
                                                                SchedWs ws, int32_t* __restrict__ center_order,
                                                                int32_t* __restrict__ pack_order,
                                                                int32_t* __restrict__ pack_ptr,
                                                                int4* __restrict__ info) {
  __shared__ int mb[kSchedWin];
  const int lane = threadIdx.x;
  const int64_t a0 = static_cast<int64_t>(kSchedWin) * blockIdx.x;
  const int na = static_cast<int>(N - a0 < kSchedWin ? N - a0 : kSchedWin);
  const int64_t s = a0 + lane;
  int d = 0;
  if (lane < na) {
    d = min(rowptr[s + 1] - rowptr[s], kSchedDeg);
    center_order[ws.apre[d] + atomicAdd(&ws.acur[d], 1)] = static_cast<int32_t>(s);
    const int tu = ws.t_unit[s];
    if (tu >= 0) {  // lane u < nu: unit u of the window
      const int key = tu >> 16, mem = tu & 0xff;
      const unsigned long long cur = atomicAdd(&ws.ucur[key], (1ull << 32) | static_cast<unsigned long long>(mem));
      const int mbase = ws.mpre[key] + static_cast<int>(cur & 0xffffffffull);
      pack_ptr[ws.upre[key] + static_cast<int>(cur >> 32)] = mbase;
      mb[lane] = mbase;
    }
  }
  __syncthreads();
  if (lane < na) {
    const int a = ws.t_order[s], pu = ws.t_posu[s];
    const int pos = mb[pu >> 8] + (pu & 0xff);
    const int r = rowptr[a], da = rowptr[a + 1] - r;
    pack_order[pos] = a;
    info[pos] = make_int4(a, r, da, (src_row && da > 0) ? src_row[r] : 0);
  }
}

}  // namespace x2g

// collate's center-kernel units on the HOST (data.center_packs; no device work): the atoms by decreasing
// degree (ties by index) packed best-fit into units of <= cap rows and <= max_members atoms — for each
// atom the fullest open unit that takes it (the most recently opened of equally full ones), a new unit
// when none does, an atom of degree >= cap alone; atoms without edges max_members to a unit, in index
// order, after all others.  Units in the order they were opened (so by decreasing largest degree).
// The Python loop this replaces took 2/3 of a 128-molecule collate.
X2G_API int x2g_center_packs_host(const int64_t* deg, int64_t n, int32_t cap, int32_t max_members, int32_t* order,
                                  int32_t* packs, int64_t* n_units, int32_t* max_rows) {
  if (n < 0 || cap < 1 || max_members < 1 || !n_units || !max_rows || n > 0x7fffffff) return X2G_EINVAL;
  if (n > 0 && (!deg || !order || !packs)) return X2G_EINVAL;
  std::vector<int32_t> idx(static_cast<size_t>(n));
  std::iota(idx.begin(), idx.end(), 0);
  std::stable_sort(idx.begin(), idx.end(), [&](int32_t x, int32_t y) { return deg[x] > deg[y]; });
  std::vector<std::vector<int32_t>> units, free_(static_cast<size_t>(cap));
  std::vector<int64_t> rows;
  for (const int32_t a : idx) {
    const int64_t d = deg[a];
    if (d <= 0) break;  // (sorted: the rest have no edges either)
    if (d < cap) {
      bool placed = false;
      for (int64_t r = d; r < cap && !placed; ++r) {
        auto& fr = free_[static_cast<size_t>(r)];
        if (fr.empty()) continue;
        const int32_t u = fr.back();
        fr.pop_back();
        units[u].push_back(a);
        rows[u] += d;
        if (static_cast<int32_t>(units[u].size()) < max_members) free_[static_cast<size_t>(r - d)].push_back(u);
        placed = true;
      }
      if (placed) continue;
      free_[static_cast<size_t>(cap - d)].push_back(static_cast<int32_t>(units.size()));
    }
    units.push_back({a});
    rows.push_back(d);
  }
  std::vector<int32_t> zero;
  for (int64_t a = 0; a < n; ++a)
    if (deg[a] <= 0) zero.push_back(static_cast<int32_t>(a));
  for (size_t i = 0; i < zero.size(); i += static_cast<size_t>(max_members)) {
    const size_t e = std::min(zero.size(), i + static_cast<size_t>(max_members));
    units.emplace_back(zero.begin() + i, zero.begin() + e);
    rows.push_back(0);
  }
  int64_t pos = 0, mr = 0;
  if (packs) packs[0] = 0;
  for (size_t u = 0; u < units.size(); ++u) {
    for (const int32_t a : units[u]) order[pos++] = a;
    packs[u + 1] = static_cast<int32_t>(pos);
    mr = std::max(mr, rows[u]);
  }
  *n_units = static_cast<int64_t>(units.size());
  *max_rows = static_cast<int32_t>(mr);
  return X2G_OK;
}

X2G_API size_t x2g_center_schedule_workspace(int64_t num_atoms) {
  return num_atoms < 0 ? 0 : (x2g::kSchedTempWord + 3 * static_cast<size_t>(num_atoms)) * sizeof(int32_t);
}

X2G_API int x2g_center_schedule(const int32_t* atom_rowptr, const int32_t* src_row, int64_t num_atoms,
                                int32_t* center_order, int32_t* pack_order, int32_t* pack_ptr, int32_t* atom_info,
                                void* workspace, size_t ws_bytes, void* stream) {
  using namespace x2g;
  if (num_atoms < 0 || num_atoms > 0x7fffffff - kSchedWin) return X2G_EINVAL;
  if (ws_bytes < x2g_center_schedule_workspace(num_atoms) || !workspace) return X2G_EWORKSPACE;
  if (num_atoms == 0) return X2G_OK;
  if (!atom_rowptr || !center_order || !pack_order || !pack_ptr || !atom_info) return X2G_EINVAL;
  if (reinterpret_cast<uintptr_t>(atom_info) % 16 || reinterpret_cast<uintptr_t>(workspace) % 8)
    return X2G_EUNSUPPORTED;
  hipStream_t st = as_stream(stream);
  const SchedWs ws = sched_ws(workspace, num_atoms);
  const hipError_t e = hipMemsetAsync(workspace, 0, kSchedApreWord * sizeof(int32_t), st);
  if (e != hipSuccess) return static_cast<int>(e);
  center_pack_window_kernel<<<static_cast<unsigned>((num_atoms + kSchedWin - 1) / kSchedWin), kSchedWin, 0, st>>>(
      atom_rowptr, num_atoms, ws);
  if (int rc = last_launch_status()) return rc;
  center_sched_scan_kernel<<<1, 256, 0, st>>>(num_atoms, ws, pack_ptr);
  if (int rc = last_launch_status()) return rc;
  center_sched_place_kernel<<<static_cast<unsigned>((num_atoms + kSchedWin - 1) / kSchedWin), kSchedWin, 0, st>>>(
      atom_rowptr, src_row, num_atoms, ws, center_order, pack_order, pack_ptr, reinterpret_cast<int4*>(atom_info));
  return last_launch_status();
}
