"""Benchmark: X2-GNN training step (molecules/s, fwd+bwd) on synthetic QM9-U0-shaped molecules.

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

One step = the reference trainer's step (trainer.py:37-48) on one resident batch of 128
molecules per GPU: xgnn_poly forward (GPU triplet build, basis, 4 SBF-transformer layers,
readouts), smooth-L1 loss, backward, one RCCL all-reduce of the flat gradient bucket (N>1),
grad-norm clip (max 100), Adam step and the EMA update.  Weak scaling: every rank owns its own
128 molecules.  Rank 0 prints ONE JSON line (contract in the task statement); besides the
metric it carries the dominant kernel's roofline (HIP-event timed here, on the stream it runs
on) and the CPU baseline (the oracle restatement, torch-CPU, on a bounded sample).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))

import x2gnn  # noqa: E402
from x2gnn import _lib, ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.dist import collate_shard, shard_by_triplets  # noqa: E402
from x2gnn.train import Inference, Trainer  # noqa: E402
from x2gnn.datasets import ATOMWISE_TARGETS, LABELS, model_for_target  # noqa: E402
from x2gnn.synth import molecules_from_geometry_file, synthetic_molecules  # noqa: E402

CFG = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)  # config.json
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MFMA_F32_PEAK_TFS = 157.3  # dense fp32 MFMA (v_mfma_f32_32x32x2_f32) peak, MI355X_MICROARCH.md
# scripts/pmc_traffic.py outputs (rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench), per workload
# the committed PMC summaries (scripts/pmc_traffic.py over rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
# this bench at the same workload and shape): bytes of each probe's own launch
TRAFFIC_JSON = {("qm9_u0", "S160"): os.path.join(ROOT, "profiles", "r6_pmc_traffic.json"),
                ("qm9_u0", "S5A"): os.path.join(ROOT, "profiles", "r6_pmc_traffic_s5a.json"),
                ("qm9_allprop", "S160"): os.path.join(ROOT, "profiles", "r6_pmc_traffic_c3.json"),
                ("aid_infer", "S160"): os.path.join(ROOT, "profiles", "r6_pmc_traffic_c5.json")}
# the config-2 step's per-kernel work table (scripts/step_work.py: PMC HBM bytes, matrix FLOPs, trace time
# per step) behind `step_roofline`
STEP_WORK_JSON = os.path.join(ROOT, "profiles", "r6_step_work.json")


def product_digest():
    """sha256 over the product sources (x2-gnn_amd/csrc/* and x2-gnn_amd/x2gnn/*.py, sorted by name): what a
    committed measurement table was taken on (.git does not travel to the GPU box, so the commit alone
    cannot be checked there)."""
    import hashlib

    h = hashlib.sha256()
    pkg = os.path.join(ROOT, "x2-gnn_amd")
    for sub, ext in (("csrc", ""), ("x2gnn", ".py")):
        d = os.path.join(pkg, sub)
        for f in sorted(os.listdir(d)):
            if f.endswith(ext) and os.path.isfile(os.path.join(d, f)):
                h.update(f"{sub}/{f}\0".encode())
                h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()


def step_roofline(ms_per_step, workload, shape):
    """The step against its own bound: every kernel of the step at its own roofline, back to back —
    sum_k max(FLOP_k / f32 MFMA peak, HBM bytes_k / HBM peak) — over the measured step time.  FLOP_k are
    the MFMA kernels' matrix FLOPs, bytes_k the PMC-measured HBM traffic per step (the committed
    table, scripts/step_work.py); VALU work (attention, elementwise) is priced by its bytes alone.  The
    table is used only when it was measured on these product sources (its digest equals
    product_digest()): a table from older sources gives {"stale": ...} instead of a fraction."""
    if workload != "qm9_u0" or shape != "S160" or not os.path.exists(STEP_WORK_JSON):
        return None
    tab = json.load(open(STEP_WORK_JSON))
    src = os.path.relpath(STEP_WORK_JSON, ROOT)
    if tab["meta"].get("digest") != product_digest():
        return {"frac": None, "stale": f"{src} was measured on other product sources (commit "
                                       f"{tab['meta'].get('commit')}): not stated", "source": src}
    rows = []
    for k, v in tab["kernels"].items():
        t_f = v["flops"] / (MFMA_F32_PEAK_TFS * 1e12) * 1e3
        t_b = v["hbm_bytes"] / (HBM_PEAK_GBS * 1e9) * 1e3
        rows.append((k, max(t_f, t_b), t_f, t_b, v["us"] * 1e-3))
    bound = sum(r[1] for r in rows)
    rows.sort(key=lambda r: -(r[4] - r[1]))
    return {"frac": round(bound / ms_per_step, 4), "bound_ms": round(bound, 4), "ms_per_step": ms_per_step,
            "mfma_ms": round(sum(r[2] for r in rows), 4), "hbm_ms": round(sum(r[3] for r in rows), 4),
            "kernel_ms_traced": round(sum(r[4] for r in rows), 4),
            "largest_gaps": [{"kernel": r[0], "traced_ms": round(r[4], 4), "bound_ms": round(r[1], 4)}
                             for r in rows[:6]],
            "source": src, "commit": tab["meta"].get("commit"), "digest": tab["meta"]["digest"][:12]}


# probe name -> the kernel (substring of its symbol) whose PMC bytes it is
PMC_KERNEL = {"sbf_project": "sbf_project_waves", "attn_fwd": "attn_fwd_center",
              "attn_bwd": "attn_bwd_center_kernel",
              "attn_bwd_dst": "attn_bwd_dst_g_batched", "attn_bwd_src": "attn_bwd_src_fold_batched",
              "sbf_radial_wgrad": "sbf_radial_wgrad"}
METRIC = "molecules/sec (fwd+bwd) on QM9 U0, batch=128, 1/2/4/8 MI355X"
AID_GEOM = os.path.join(ROOT, "tests", "golden", "aid_geom.npz")  # raw/AID_kcal.xyz as arrays
# BASELINE.json configs: [1] is the metric's; [2] and [4] are the other single-GPU shapes
WORKLOADS = {
    "qm9_u0": dict(batch=128, train=True, metric=METRIC),
    "qm9_allprop": dict(batch=256, train=True,
                        metric="molecules/sec (fwd+bwd) on QM9 all-property target model, batch=256, MI355X"),
    "aid_infer": dict(batch=64, train=False,
                      metric="molecules/sec (inference) on AID_kcal (~83 atoms), batch=64, MI355X"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="molecules per GPU (default: the workload's)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="molecules per step over all ranks (default: gpus x batch; BASELINE config 4 = 1024 "
                         "over 8); one global batch, sharded by triplet count (x2gnn.dist.shard_by_triplets)")
    ap.add_argument("--shape", default="S160", choices=["S160", "S5A"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-loader", action="store_true", help="skip the fresh-batch DataLoader side field")
    ap.add_argument("--no-lazy-sbf", action="store_true", help="write the [T, 42] sbf rows (ops.LAZY_SBF False)")
    ap.add_argument("--device-schedule", action="store_true",
                    help="collate without the center schedule: the step makes it on the device (data.HOST_SCHEDULE)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the step")
    ap.add_argument("--workload", default="qm9_u0", choices=sorted(WORKLOADS),
                    help="qm9_u0: BASELINE config 2 (the metric); qm9_allprop: config 3 (one target's model, "
                         "B=256); aid_infer: config 5 (AID_kcal geometries, B=64, inference)")
    ap.add_argument("--target", type=int, default=0, help="qm9_allprop: QM9 target 0-11 (train_ema.py:41-44)")
    ap.add_argument("--step-only", action="store_true",
                    help="A/B runs: print only the timed-step line fields (no kernel probes, no CPU baseline)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1: nccl (= RCCL over xGMI, the measured path); gloo only rehearses the "
                         "multi-rank step on a box with fewer GPUs than ranks")
    args = ap.parse_args()
    w = WORKLOADS[args.workload]
    if args.batch is None:
        args.batch = w["batch"]
    return args


# ------------------------------------------------------------------------------------------ kernels
def attention_probe(model, batch, reps, train=True):
    """Time the fused attention kernels of conv layer 0 on this step's real inputs with HIP
    events on the launch stream; returns {kernel: (avg_ms, algorithmic_bytes_per_launch)}.  ``train``
    False: the forward as inference runs it (no logits, no S / P rows stored)."""
    conv = model.fin_model.convs[0]
    line, plan = model.line_graph_data(batch)  # grad mode on: keeps the sbf factors (rbf_env, Y)
    lg = plan.lg
    _, radial, ylm = lg.sbf_factors
    with torch.no_grad():
        x, rbf, sbf = line.x, line.node_rbf, line.edge_sbf
        table = conv.lin_edge(model.fin_model.edgenn(line.edge_attr)).contiguous()
        row = plan.dst_type
        x_src = x * conv.lin_rbf(rbf)
        q, k, v = conv.lin_query(x), conv.lin_key(x_src), conv.lin_value(x_src)
        skip = conv.lin_skip(x)
    E, T, H, C = lg.E, lg.T, conv.heads, conv.out_channels
    D = H * C
    W, bsb = conv.lin_sbf.weight.detach().contiguous(), conv.lin_sbf.bias.detach().contiguous()
    f32 = dict(dtype=torch.float32, device=x.device)
    out = torch.empty(E, D, **f32)
    alpha, smax, sden = torch.empty(T, H, **f32), torch.empty(E, H, **f32), torch.empty(E, H, **f32)
    dout = torch.randn(E, D, **f32)
    dq, dk, dv, dedge = (torch.empty(E, D, **f32) for _ in range(4))
    dlogit, dproj = torch.empty(T, H, **f32), torch.empty(T, D, **f32)
    src_rowptr, src_perm = lg.src_csr()
    S = sbf.shape[1]

    sproj = torch.empty(T, D, **f32)

    def proj():
        call("x2g_sbf_project", ptr(sbf), T, S, ptr(W), ptr(bsb), D, ptr(sproj), stream_ptr())

    proj()  # the model's path: S = lin_sbf(sbf) once per layer, kernels read S rows (weight NULL)

    def fwd():
        call("x2g_sbf_attention_fwd", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(row), ops.EDGE_PER_DST,
             ptr(sproj), None, None, ptr(lg.trip_rowptr), ptr(lg.trip_src), E, T, H, C, D, ptr(out), ptr(alpha),
             ptr(smax), ptr(sden), stream_ptr())

    prob, rho = torch.empty(T, H, **f32), torch.empty(E, H, **f32)
    gfold = torch.empty(E, 8, D, **f32)
    dwr, dbr = torch.empty(D, S, **f32), torch.empty(D, **f32)
    ws_bytes = int(_lib.load().x2g_sbf_radial_wgrad_workspace(E, D))
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)

    def bwd_dst():  # the factorised backward the model runs (csrc/attention_fold.inc)
        call("x2g_sbf_attention_bwd_dst_g", ptr(q), ptr(k), ptr(v), ptr(table), ptr(row), ops.EDGE_PER_DST,
             ptr(sproj), ptr(lg.trip_rowptr), ptr(lg.trip_src), ptr(alpha), ptr(smax), ptr(sden), ptr(dout), E, T, H,
             C, ptr(dq), ptr(dedge), None if ops._SRC_G else ptr(dlogit), ptr(prob), ptr(rho), stream_ptr())

    def bwd_src():
        call("x2g_sbf_attention_bwd_src_fold", ptr(q), ptr(v), ptr(table), ptr(row), ptr(lg.src_type),
             table.shape[0], ops.EDGE_PER_DST, ptr(sproj), ptr(ylm), ptr(src_rowptr), ptr(src_perm), ptr(lg.src_dst),
             ptr(lg.trip_dst), ptr(prob), None if ops._SRC_G else ptr(dlogit), ptr(rho), ptr(dout), E, T, H, C, ptr(dk),
             ptr(dv), ptr(gfold), stream_ptr())

    def radial_wgrad():
        call("x2g_sbf_radial_wgrad", ptr(gfold), ptr(radial), E, D, ptr(dwr), ptr(dbr), 0, ptr(ws), ws_bytes,
             stream_ptr())

    center, src_row = ops._center_rows(lg, ops.EDGE_PER_DST, row, D, C)
    center_bwd = center and ops._CENTER_BWD and lg.atom_type is not None
    atom_de = torch.empty(lg.N, D, **f32)
    g_work = torch.empty(2, T, H, **f32)

    def fwd_center():  # the model's forward on a symmetric line graph (csrc/attention_center.hip)
        call("x2g_sbf_attention_fwd_center", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(src_row),
             ops.EDGE_PER_DST, ptr(sproj), 0, ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip),
             ptr(lg.center_order), 0, lg.N, lg.max_degree, E, T, H, C, ptr(out), ptr(alpha), ptr(smax), ptr(sden),
             None, stream_ptr())

    sf = center and ops._center_sf_ok(lg, (radial, ylm), D)

    # the model's units: the leading hub units (atoms beyond the fused forward's LDS image) source-tiled, the rest
    # untiled (ops._center_split)
    order, packs, info, launches = ops._center_split(lg) if center else (None, None, None, [])

    # as the model: with the fused forward feeding the center backward, P rows [E, 7, D] pass between them
    # instead of S rows [T, D] (ops._CENTER_P)
    use_p = sf and center_bwd and ops._CENTER_P
    pbuf = torch.empty(E, 7, D, **f32) if use_p else None

    def fwd_sf():  # the model's forward with lin_sbf fused (S rebuilt per workgroup unit; P or S rows stored)
        common = (ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(src_row), ops.EDGE_PER_DST, ptr(radial), ptr(ylm),
                  ptr(W), ptr(bsb), ptr(lg.atom_rowptr), ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(order), ptr(packs),
                  ptr(info))
        if train:
            outs = (E, T, H, C, ptr(out), ptr(alpha), ptr(smax), ptr(sden), None, None if use_p else ptr(sproj),
                    ptr(pbuf), stream_ptr())
        else:  # inference (ops.sbf_attention without attention weights): nothing for a backward
            outs = (E, T, H, C, ptr(out), None, ptr(smax), ptr(sden), None, None, None, stream_ptr())
        ops._center_launch(launches, common, outs)

    def bwd_center():  # both backward passes in one launch per center atom
        call("x2g_sbf_attention_bwd_center", ptr(q), ptr(k), ptr(v), ptr(table), ptr(src_row), ops.EDGE_PER_DST,
             None if use_p else ptr(sproj), ptr(pbuf), ptr(bsb) if use_p else None, ptr(ylm), ptr(lg.atom_rowptr),
             ptr(lg.edge_rev), ptr(lg.rev_trip), ptr(lg.center_order),
             ptr(alpha), ptr(smax), ptr(sden), ptr(dout), lg.N, lg.max_degree, E, T, H, C, ptr(dq), ptr(dk),
             ptr(dv), ptr(gfold), ptr(atom_de), ptr(g_work), stream_ptr())

    row_b = 4 * D
    # Bytes per launch, two ways.  "bytes" (the roofline's algorithmic figure): every array the
    # kernel needs, each element once -- k / v / q / dout rows count once per LINE NODE however
    # many triplets gather them, so a kernel at HBM speed cannot exceed the 8 TB/s peak.
    # "gathered_bytes": every row fetch as issued (k / v rows once per triplet), i.e. the load
    # the cache hierarchy serves; informative only, no GB/s is quoted for it.  The PMC-measured
    # HBM bytes (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, profiles/*_pmc_traffic.json) sit beside both.
    idx = 4 * T + 4 * (E + 1)  # one CSR (ids + row pointers)
    proj_bytes = T * (4 * S + row_b) + 4 * D * (S + 1)
    fwd_bytes = idx + T * (row_b + 4 * H) + E * (4 + 5 * row_b + 8 * H)  # q k v skip out, S, alpha, max/den
    fwd_gath = idx + T * (3 * row_b + 4 * H) + E * (4 + 3 * row_b + 8 * H)
    gh = 0 if ops._SRC_G else 4 * H  # g [T, H]: written by the destination pass, read by the source pass
    dst_bytes = idx + T * (row_b + 8 * H + gh) + E * (4 + 6 * row_b + 12 * H)  # q k v dout dq d_edge, S, a/p(/g)
    dst_gath = idx + T * (3 * row_b + 8 * H + gh) + E * (4 + 4 * row_b + 12 * H)
    # source-major CSR + src_dst; S and Y rows, prob (, g); q v dout read, dk dv written, G [E, 8, D]
    src_bytes = idx + 4 * T + T * (row_b + 32 + 4 * H + gh) + E * (4 + 13 * row_b + 4 * H)
    src_gath = idx + 4 * T + T * (3 * row_b + 32 + 4 * H + gh) + E * (4 + 11 * row_b + 4 * H)
    radial_bytes = E * (8 * row_b + 4 * S) + 4 * D * (S + 1)
    # center-atom kernels: every row once (k / v staged per atom, not gathered per triplet); indices are
    # atom_rowptr, edge_rev, rev_trip and the per-source element row
    cidx = 4 * (lg.N + 1) + 12 * E
    cfwd_bytes = cidx + T * (row_b + 4 * H) + E * (5 * row_b + 8 * H)  # k v q skip out, S, alpha, max/den
    # reads k v q dout, S rows (or the P rows), alpha, Y, max/den; writes dq dk dv, G [E, 8, D], the per-atom
    # edge gradient (the (g, a) scratch, written once and read back from L2 by the same workgroup, not counted)
    s_or_p = E * 7 * row_b + 4 * D if use_p else T * row_b
    cbwd_bytes = (cidx + T * (4 * H + 32) + s_or_p + E * (4 * row_b + 8 * H) + E * (3 * row_b + 8 * row_b)
                  + lg.N * row_b)
    # fused projection: k v q skip out rows, the radial rows and the weight, Y, alpha, max/den, S (or P) rows
    # written
    sf_bytes = cidx + T * (4 * H + 32) + (E * 7 * row_b if use_p else T * row_b) + E * (5 * row_b + 8 * H + 4 * S) \
        + 4 * D * (S + 1)
    if not train:  # Y rows in, out / max / den out: no logits, no S or P rows
        sf_bytes = cidx + T * 32 + E * (5 * row_b + 8 * H + 4 * S) + 4 * D * (S + 1)
    probes = [] if sf else [("sbf_project", proj, proj_bytes, proj_bytes)]
    if sf:
        probes.append(("attn_fwd", fwd_sf, sf_bytes, sf_bytes))
    elif center:
        probes.append(("attn_fwd", fwd_center, cfwd_bytes, cfwd_bytes))
    else:
        probes.append(("attn_fwd", fwd, fwd_bytes, fwd_gath))
    if center_bwd:
        probes.append(("attn_bwd", bwd_center, cbwd_bytes, cbwd_bytes))
    else:
        probes += [("attn_bwd_dst", bwd_dst, dst_bytes, dst_gath), ("attn_bwd_src", bwd_src, src_bytes, src_gath)]
    probes.append(("sbf_radial_wgrad", radial_wgrad, radial_bytes, radial_bytes))
    res = {}
    for name, fn, nbytes, gath in probes:
        res[name] = (_event_time(fn, reps), nbytes, gath)
    return res, dict(E=E, T=T, D=D, center=center, center_bwd=center_bwd, sf=sf)


def dense_probe(R, reps):
    """The trunk's dense layer at this step's row count: [R,128] x [128,128] + bias, SiLU and
    residual fused (x2g_dense_fwd), and its fused backward (x2g_dense_bwd: dz, dx, dW, db =
    dense_bwd_persist + the fixed-order slab sum), HIP-event timed on the launch stream."""
    K = N = 128
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(R, K, device=dev, generator=g)
    w = 0.1 * torch.randn(N, K, device=dev, generator=g)
    b = torch.randn(N, device=dev, generator=g)
    dy = torch.randn(R, N, device=dev, generator=g)
    y, z, dx = (torch.empty(R, N, device=dev) for _ in range(3))
    dw, db = torch.empty(N, K, device=dev), torch.empty(N, device=dev)
    wsb = _lib_ws("x2g_dense_bwd_workspace", R, K, N)
    ws = torch.empty(max(wsb, 4) // 4 + 1, device=dev)

    def fwd():
        call("x2g_dense_fwd", ptr(x), ptr(w), ptr(b), R, K, N, ops.ACT_SILU, ptr(x), ptr(y), ptr(z), stream_ptr())

    def bwd():
        call("x2g_dense_bwd", ptr(dy), ptr(z), ops.ACT_SILU, ptr(x), ptr(w), R, K, N, ptr(dx), ptr(dw), ptr(db),
             ptr(ws), wsb, stream_ptr())

    fwd()
    return {"dense_fwd": (_event_time(fwd, reps), 2.0 * R * K * N), "dense_bwd": (_event_time(bwd, reps), 4.0 * R * K * N)}


def chain_probe(R, reps, mol_rows=165):
    """The trunk tail as the step runs it (ops.row_chain, model.py:47-50: 7 Linear stages per conv
    layer) at this step's row count: x2g_chain_fwd_ln (the graph LayerNorm of model.py:46 applied
    while staging, molecules of ``mol_rows`` line nodes, with the T-layout stage inputs),
    x2g_chain_bwd_ln (T-layout dz, the residual gradient accumulated into the layer input's fan-in
    buffer as the trunk does, the LayerNorm's per-row sums) and x2g_chain_wgrad (slab sums deferred,
    as in the step), HIP-event timed on the launch stream.  FLOPs per launch: 7 * 2 * R * 128 * 128
    each (the LayerNorm's are not counted)."""
    D, n = 128, 7
    S, H, RH, RE = ops.CHAIN_SILU, ops.CHAIN_HOLD, ops.CHAIN_RES_HELD, ops.CHAIN_RES_EXT
    flags = [S | H, S | RH, S | RE, S | H, S | RH, S | H, S | RH]
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(4)
    x, res, dy = (torch.randn(R, D, device=dev, generator=g) for _ in range(3))
    W = [torch.randn(D, D, device=dev, generator=g) / 11.3 for _ in range(n)]
    B = [0.1 * torch.randn(D, device=dev, generator=g) for _ in range(n)]
    Z = [torch.empty(R, D, device=dev) for _ in range(n)]
    y, dx = (torch.empty(R, D, device=dev) for _ in range(2))
    dres = torch.zeros(R, D, device=dev)  # accumulated into (RES_ACCUM), as the fan-in buffer is
    WT = torch.empty(n, D, D, device=dev)
    tf = _lib_ws("x2g_chain_t_floats", R, D)
    in_t, dz_t = torch.empty(n, tf, device=dev), torch.empty(n, tf, device=dev)
    DW = [torch.empty(D, D, device=dev) for _ in range(n)]
    DB = [torch.empty(D, device=dev) for _ in range(n)]
    st = (ops.ChainStage * n)(*[ops.ChainStage(W[i].data_ptr(), B[i].data_ptr(), Z[i].data_ptr(),
                                               y.data_ptr() if i == n - 1 else None, WT[i].data_ptr(), flags[i])
                                for i in range(n)])
    bflags = [f | (ops.CHAIN_RES_ACCUM if f & RE else 0) for f in flags]
    bst = (ops.ChainBwdStage * n)(*[ops.ChainBwdStage(W[i].data_ptr(), WT[i].data_ptr(), Z[i].data_ptr(), None,
                                                      bflags[i]) for i in range(n)])
    ptr_np = np.unique(np.concatenate([np.arange(0, R, mol_rows), [R]])).astype(np.int32)
    seg = torch.from_numpy(ptr_np).to(dev)
    G = len(ptr_np) - 1
    xm = x.mean(1)
    stats = torch.stack([xm, ((x - xm[:, None]) ** 2).sum(1)], 1).contiguous()
    xn, rstd, gst = torch.empty(R, D, device=dev), torch.empty(G, device=dev), torch.empty(R, 2, device=dev)
    wsb = _lib_ws("x2g_chain_wgrad_workspace", R, D, n)
    ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    dwa = (ctypes.c_void_p * n)(*[t.data_ptr() for t in DW])
    dba = (ctypes.c_void_p * n)(*[t.data_ptr() for t in DB])

    def fwd():
        call("x2g_chain_fwd_ln", ptr(x), ptr(stats), ptr(seg), G, 1e-8, ptr(xn), None, ptr(rstd), ptr(res), st, n,
             R, D, ptr(in_t), stream_ptr())

    def bwd():
        call("x2g_chain_bwd_ln", ptr(dy), None, bst, n, R, D, ptr(dx), ptr(dres), ptr(dz_t), ptr(xn), ptr(gst),
             stream_ptr())

    def wgrad():
        call("x2g_chain_wgrad", ptr(in_t), ptr(dz_t), n, R, D, dwa, dba, ops.DEFER_SLAB_SUM, ptr(ws), wsb, stream_ptr())

    fwd()
    bwd()
    flops = 2.0 * n * R * D * D
    return {"chain_fwd": (_event_time(fwd, reps), flops), "chain_bwd": (_event_time(bwd, reps), flops),
            "chain_wgrad": (_event_time(wgrad, reps), flops)}


def proj_probe(R, reps):
    """The conv projections as the step runs them at this row count: x2g_conv_proj_fwd (lin_rbf
    gate + q, k, v, skip, the T-layout x / x_src and W^T) and x2g_conv_proj_bwd_gate (dx, the gate's
    drbf and dW_rbf slab, the four T-layout output gradients), HIP-event timed on the launch stream.
    FLOPs per launch: 4 * 2 * R * 128 * 128 each."""
    D, RR = 128, 6
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(6)
    x = torch.randn(R, D, device=dev, generator=g)
    rbf = torch.randn(R, RR, device=dev, generator=g)
    wr = torch.randn(D, RR, device=dev, generator=g)
    W = [torch.randn(D, D, device=dev, generator=g) / 11.3 for _ in range(4)]
    B = [torch.randn(D, device=dev, generator=g) for _ in range(4)]
    out = [torch.empty(R, D, device=dev) for _ in range(4)]
    grads = [torch.randn(R, D, device=dev, generator=g) for _ in range(4)]
    WT = [torch.empty(D, D, device=dev) for _ in range(4)]
    tf = _lib_ws("x2g_chain_t_floats", R, D)
    x_t, xs_t = torch.empty(tf, device=dev), torch.empty(tf, device=dev)
    g_t = [torch.empty(tf, device=dev) for _ in range(4)]
    dx, drbf, dw = torch.zeros(R, D, device=dev), torch.empty(R, RR, device=dev), torch.empty(D, RR, device=dev)
    wsb = _lib_ws("x2g_conv_proj_bwd_gate_workspace", R, RR)
    ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    proj = (ops.Proj * 4)(*[ops.Proj(W[p].data_ptr(), B[p].data_ptr(), out[p].data_ptr(), WT[p].data_ptr())
                            for p in range(4)])
    pg = (ops.ProjGrad * 4)(*[ops.ProjGrad(grads[p].data_ptr(), W[p].data_ptr(), WT[p].data_ptr(),
                                           g_t[p].data_ptr()) for p in range(4)])

    def fwd():
        call("x2g_conv_proj_fwd", ptr(x), ptr(rbf), RR, ptr(wr), proj, R, D, ptr(x_t), ptr(xs_t), stream_ptr())

    def bwd():  # dx += (the fan-in form the step uses after the first consumer)
        call("x2g_conv_proj_bwd_gate", pg, R, D, ptr(x), ptr(rbf), RR, ptr(wr), ptr(dx), ptr(dx), ptr(drbf),
             ptr(dw), 0, ptr(ws), wsb, stream_ptr())

    fwd()
    flops = 4 * 2.0 * R * D * D
    return {"conv_proj_fwd": (_event_time(fwd, reps), flops), "conv_proj_bwd_gate": (_event_time(bwd, reps), flops)}


def flat_wgrad_probe(flat_launches, reps):
    """The step's largest kernel: every T-layout weight gradient of the backward in one launch
    (x2g_tiled_wgrad_flat_rows, ops._flush_tiled) with the job list the captured step recorded
    (Trainer.flat_launches: per job its rows R_j and one [128, cols_j] dW = dz^T x, K = R_j — the trunk's
    line-node rows and the readout MLPs' atom rows in the same launch), on synthetic T-layout operands,
    HIP-event timed on the launch stream.  FLOPs per launch: sum_j 2 * R_j * 128 * cols_j."""
    if not flat_launches:
        return None
    launch = max(flat_launches, key=lambda l: sum(R * c for R, c in l))
    n, D = len(launch), 128
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(5)
    x_t, dz_t = [], []
    for R, _ in launch:
        tf = _lib_ws("x2g_chain_t_floats", R, D)
        x_t.append(torch.randn(tf, device=dev, generator=g))
        dz_t.append(torch.randn(tf, device=dev, generator=g))
    dw = [torch.zeros(D, D, device=dev) for _ in range(n)]
    db = [torch.zeros(D, device=dev) for _ in range(n)]
    jobs = (ops.TiledJob * n)(*[ops.TiledJob(dz_t[j].data_ptr(), x_t[j].data_ptr(), dw[j].data_ptr(),
                                             db[j].data_ptr(), D if c < D else 0, c if c < D else 0)
                                for j, (_, c) in enumerate(launch)])
    rows = (ctypes.c_int64 * n)(*[R for R, _ in launch])
    from x2gnn import _lib
    wsb = int(_lib.load().x2g_tiled_wgrad_flat_rows_workspace(rows, n, D))
    ws = torch.empty(max(wsb, 4), dtype=torch.uint8, device=dev)
    out = (ops.SlabJob * n)()

    def run():
        call("x2g_tiled_wgrad_flat_rows", jobs, rows, n, D, ops.ACCUM_WGRAD | ops.DEFER_SLAB_SUM, out, ptr(ws), wsb,
             stream_ptr())

    run()
    ms = _event_time(run, reps)
    tiles = sum((R + 15) // 16 for R, _ in launch)
    wgs = min(512, max(1, tiles))  # chain.hip flat_grid: two 512-thread workgroups per CU
    return {"ms": ms, "flops": float(sum(2.0 * R * D * c for R, c in launch)),
            "rows": sorted({R for R, _ in launch}), "jobs": n, "grid": wgs * 512}


def in_step_kernel_ms(runner, batch, name, reps):
    """The named kernel's duration INSIDE the training step: ``reps`` eager forward+backward passes
    with HIP events around that launch on its stream (ops.KERNEL_TIMERS: a sleep kernel ahead of the
    start event keeps the device busy while the host enqueues the launch), median over passes.  The
    operands are the ones the same backward just wrote (MALL-warm), as in the captured step."""
    ops.KERNEL_TIMERS[name] = []
    try:
        for _ in range(reps):
            runner.forward_backward(batch)
        torch.cuda.synchronize()
        evs = ops.KERNEL_TIMERS[name]
    finally:
        ops.KERNEL_TIMERS.pop(name, None)
    runner.bucket.zero()
    ms = sorted(a.elapsed_time(b) for a, b in evs)
    return (ms[len(ms) // 2], len(ms)) if ms else (None, 0)


def _lib_ws(name, *args):
    from x2gnn import _lib

    return int(getattr(_lib.load(), name)(*args))


def load_traffic(workload, shape="S160"):
    """(path, {"<kernel>|<grid>": {"fetch_bytes", "write_bytes", ...}}) of the committed PMC summary
    for this workload and shape, or (path, None)."""
    path = TRAFFIC_JSON.get((workload, shape))
    if path is None or not os.path.exists(path):
        return path, None
    return path, json.load(open(path))["kernels"]


def pmc_traffic(keys, table):
    """HBM bytes per launch of the named kernels (sum over (symbol substring, grid) keys)."""
    if table is None:
        return None
    total = 0
    for name, grid in keys:
        hit = [v for k, v in table.items() if name in k.split("|")[0] and (grid is None or k.endswith("|" + grid))]
        if not hit or hit[0]["fetch_bytes"] is None or hit[0]["write_bytes"] is None:
            return None
        # several grids of one kernel (another probe's shape): the one with the most bytes is the step's
        best = max(hit, key=lambda v: v["fetch_bytes"] + v["write_bytes"])
        total += best["fetch_bytes"] + best["write_bytes"]
    return total


def _pmc_bytes(probe_name, table):
    return pmc_traffic([(PMC_KERNEL[probe_name], None)], table)


def _hbm_entry(name, v, table):
    """One probe kernel in the bench line: time, algorithmic bytes and GB/s, gathered bytes, and the
    PMC-measured HBM bytes and GB/s (None when no PMC summary covers it)."""
    ms, nbytes, gath = v
    hbm = _pmc_bytes(name, table)
    return {"ms": round(ms, 5), "bytes": int(nbytes), "GBs": round(nbytes / (ms * 1e-3) / 1e9, 1),
            "gathered_bytes": int(gath), "hbm_bytes": hbm,
            "hbm_GBs": None if hbm is None else round(hbm / (ms * 1e-3) / 1e9, 1)}


# MFMA probe name -> the kernel (symbol substring) whose PMC bytes it is
PMC_MFMA_KERNEL = {"conv_proj_fwd": "conv_proj_fwd_kernel", "conv_proj_bwd_gate": "conv_proj_bwd_gate_kernel",
                   "chain_fwd": "chain_fwd_v4_ln(", "chain_bwd": "chain_bwd_v3_batch",
                   "tiled_wgrad_flat": "tiled_flat_kernel"}


def _mfma_entry(name, v, table):
    """One MFMA probe in the bench line: time, FLOPs, TF/s and its fraction of the f32 MFMA peak,
    and the PMC-measured HBM bytes / GB/s of the same kernel in the step (when the summary has it)."""
    ms, flops = v
    tfs = flops / (ms * 1e-3) / 1e12
    e = {"ms": round(ms, 5), "flops": int(flops), "TFs": round(tfs, 2), "mfma_frac": round(tfs / MFMA_F32_PEAK_TFS, 4)}
    if name in PMC_MFMA_KERNEL:
        hbm = pmc_traffic([(PMC_MFMA_KERNEL[name], None)], table)
        e["hbm_bytes"] = hbm
        e["hbm_GBs"] = None if hbm is None else round(hbm / (ms * 1e-3) / 1e9, 1)
    return e


def _event_time(fn, reps):
    st = torch.cuda.current_stream()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    start.record(st)
    for _ in range(reps):
        fn()
    end.record(st)
    end.synchronize()
    return start.elapsed_time(end) / reps


def scatter_add_probe(lg, reps):
    """The graded CSR-by-destination scatter-add (x2g_segment_sum) at the step's line-graph
    shape: [T, 128] messages -> [E, 128], algorithmic bytes 4*T*D + 4*(E+1) + 4*E*D.
    Timed L2/MALL-warm (back-to-back) and cache-busted: 512 MiB are *read* between launches, which
    evicts L2 and the 256 MiB MALL without leaving dirty lines whose write-back would be billed
    to the timed kernel."""
    E, T, D = lg.E, lg.T, 128
    dev = lg.trip_rowptr.device
    msgs = torch.randn(T, D, device=dev)
    out = torch.empty(E, D, device=dev)
    nbytes = 4 * T * D + 4 * (E + 1) + 4 * E * D

    def fn():
        call("x2g_segment_sum", ptr(msgs), None, ptr(lg.trip_rowptr), E, D, ptr(out), stream_ptr())

    warm = _event_time(fn, reps)
    flush = torch.ones(512 * 2 ** 20 // 4, device=dev)
    sink = torch.empty((), device=dev)
    st = torch.cuda.current_stream()
    times = []
    for _ in range(reps):
        torch.sum(flush, dim=0, out=sink)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        fn()
        b.record(st)
        b.synchronize()
        times.append(a.elapsed_time(b))
    ref = torch.zeros(E, D, device=dev).index_add_(0, lg.trip_dst.long(), msgs)
    ok = torch.allclose(out, ref, rtol=1e-4, atol=1e-4)
    return dict(bytes=nbytes, warm_ms=warm, cold_ms=float(np.median(times)), parity=bool(ok))


# ------------------------------------------------------------------------------------------ cpu
CALIBRATION_JSON = os.path.join(ROOT, "profiles", "r4_cpu_calibration.json")  # scripts/calibrate_cpu_baseline.py


def host_cores():
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU quota (the GPU box
    grants each job a share of a large host; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def _time_cpu(model, b, budget_s, train, threads):
    from oracle import ref_cpu

    torch.set_num_threads(threads)
    times = []
    t_end = time.perf_counter() + budget_s
    for i in range(100):
        t0 = time.perf_counter()
        if train:
            model.zero_grad(set_to_none=True)
            res = ref_cpu.run_batch(model, b)
            torch.nn.functional.smooth_l1_loss(res, b.y).backward()
        else:
            with torch.no_grad():
                ref_cpu.run_batch(model, b)
        dt = time.perf_counter() - t0
        if i > 0:
            times.append(dt)
        if time.perf_counter() > t_end and len(times) >= 2:
            break
    return float(np.median(times)), len(times)


class _LoaderBatches(torch.utils.data.Dataset):
    """Batch i = collate of molecule group i % len(groups) (made in a DataLoader worker)."""

    def __init__(self, groups, n):
        self.groups, self.n = groups, n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return collate(self.groups[i % len(self.groups)])


def loader_probe(cfg, dev, steps=30, warm=5, workers=4, batch=128, shape="S160", groups=4):
    """End-to-end training rate with a FRESH batch every step (side field, never `value`): a torch DataLoader
    whose 4 worker processes collate molecule groups (x2gnn.data.collate, PyG's collate + the int32 index
    forms), pinned host memory, a non-blocking H2D copy, and an eager Trainer step (a new batch's sizes cannot
    replay a captured graph: each step plans its line graph and launches every kernel from the host).  Also the
    eager step on one resident batch, which bounds it."""
    from torch.utils.data import DataLoader

    mol_groups = [synthetic_molecules(batch, shape, seed=3000 + g) for g in range(groups)]
    torch.manual_seed(0)
    model = x2gnn.xgnn_poly(device="cuda", **cfg).to(dev)
    tr = Trainer(model)
    dl = DataLoader(_LoaderBatches(mol_groups, warm + steps), batch_size=None, num_workers=workers, pin_memory=True,
                    prefetch_factor=4, persistent_workers=False)
    it = iter(dl)
    for _ in range(warm):
        tr.step(next(it).to(dev, non_blocking=True))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(next(it).to(dev, non_blocking=True))
    torch.cuda.synchronize()
    t_loader = time.perf_counter() - t0
    del it, dl
    resident = collate(mol_groups[0]).to(dev)
    for _ in range(3):
        tr.step(resident)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        tr.step(resident)
    torch.cuda.synchronize()
    t_eager = time.perf_counter() - t0
    return {"value": round(batch * steps / t_loader, 2), "unit": "molecules/s", "workers": workers, "steps": steps,
            "ms_per_step": round(1e3 * t_loader / steps, 4),
            "eager_resident_ms_per_step": round(1e3 * t_eager / steps, 4),
            "note": ("end-to-end: a fresh collated batch per step from a DataLoader of 4 worker processes (pinned, "
                     "non-blocking H2D), eager Trainer step (fwd + loss + bwd + clip / Adam / EMA); not `value`, "
                     "whose batch is resident and whose step is a replayed HIP graph")}


def cpu_baseline(mols, budget_s, global_pool=None, train=True, sample=None):
    """The oracle (torch-CPU restatement of the reference) fwd+bwd (or forward only) on the same
    batch — or its first ``sample`` molecules, rate scaled per molecule — timed for ~budget_s
    seconds each at all of this host's usable cores and at 4 threads (config.json num_thread),
    plus the reference-equivalent rates from the calibration this build container recorded
    (reference / restatement speed on the same cores, scripts/calibrate_cpu_baseline.py)."""
    from oracle import ref_cpu

    prev = torch.get_num_threads()
    cores = host_cores()
    model = ref_cpu.XGNN(global_pool=global_pool, **CFG)
    full = len(mols)
    if sample is not None and sample < full:
        mols = mols[:sample]
    b = collate(mols)
    calib = json.load(open(CALIBRATION_JSON))["threads"] if os.path.exists(CALIBRATION_JSON) else {}
    legs = {}
    for threads in sorted({cores, 4}, reverse=True):
        step, n = _time_cpu(model, b, budget_s, train, threads)
        # the calibration row measured nearest this thread count (8 = the container's cores, or 4)
        row = calib.get("4" if threads <= 4 else "8")
        rate = len(mols) / step
        legs[threads] = {"value": round(rate, 2), "steps": n,
                         "reference_equivalent": (round(rate * row["reference_over_port"], 2) if row and train
                                                  else None)}
    torch.set_num_threads(prev)
    main = legs[cores]
    return {"value": main["value"], "unit": "molecules/s", "cores": cores, "kind": "port",
            "reference_equivalent": main["reference_equivalent"],
            "at_4_threads": legs[4],
            "calibration": os.path.relpath(CALIBRATION_JSON, ROOT) if calib else None,
            "sample": f"oracle/ref_cpu.py {'fwd+bwd (no optimizer)' if train else 'forward'} on "
                      f"{'the same' if len(mols) == full else f'the first {len(mols)} molecules of the'} "
                      f"{full}-molecule batch, median of {main['steps']} steps after 1 warm-up, torch-CPU fp32, "
                      f"{cores} threads = this job's usable host CPUs ({os.cpu_count()} logical CPUs on the "
                      f"machine); reference_equivalent = value x (reference / restatement speed measured on the "
                      f"same cores in the build container)"}


# ------------------------------------------------------------------------------------------ main
def main():
    args = parse()
    if args.no_lazy_sbf:
        ops.LAZY_SBF = False
    if args.device_schedule:
        import x2gnn.data as xdata

        xdata.HOST_SCHEDULE = False
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; ranks beyond the visible GPUs (a gloo rehearsal on a 1-GPU box) share them
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    torch.manual_seed(0)  # identical initial weights on every rank

    wl = WORKLOADS[args.workload]
    # one global batch of world * batch molecules (BASELINE config 4: 1024 = 8 x 128), the same on
    # every rank, sharded by triplet count (x2gnn.dist.shard_by_triplets)
    global_batch = args.global_batch if args.global_batch is not None else world * args.batch
    if args.workload == "aid_infer":  # consecutive AID molecules (wrapping), real geometries
        n_aid = int(np.load(AID_GEOM)["counts"].shape[0])
        all_mols = molecules_from_geometry_file(AID_GEOM, indices=[i % n_aid for i in range(global_batch)], seed=0)
    else:
        all_mols = synthetic_molecules(global_batch, args.shape, seed=1000)
    shards = shard_by_triplets([m["triplet_num"] for m in all_mols], world)
    mols = [all_mols[i] for i in shards[rank]]
    # the shards' triplet totals: the straggler bound of the step (every rank waits for the largest)
    shard_t = [int(sum(all_mols[i]["triplet_num"] for i in s)) for s in shards]
    host_batch, n_local, _ = collate_shard(all_mols, world, rank)
    batch = host_batch.to(dev)
    # the per-batch host cost a data loader has to hide under the step (side fields, not `value`):
    # collate (PyG Batch.from_data_list restated + the int32 index forms) and the H2D copy, warm; the median of
    # 5 each (one sample read 5 to 15 ms for config 2's collate on the same box, host noise)
    t_col, t_h2d = [], []
    for _ in range(5):
        t0 = time.perf_counter()
        host_batch, _, _ = collate_shard(all_mols, world, rank)
        t1 = time.perf_counter()
        host_batch.to(dev)
        torch.cuda.synchronize()
        t_col.append(t1 - t0)
        t_h2d.append(time.perf_counter() - t1)
    t_c0, t_c1, t_c2 = 0.0, float(np.median(t_col)), float(np.median(t_col)) + float(np.median(t_h2d))
    del host_batch, all_mols
    global_pool = None
    if args.workload == "qm9_allprop":
        model = model_for_target(args.target, CFG, device="cuda").to(dev)  # train_ema.py:41-44
        if args.target not in ATOMWISE_TARGETS:
            global_pool = "mean"
    else:
        model = x2gnn.xgnn_poly(device="cuda", **CFG).to(dev)
    runner = (Trainer(model, local_count=len(mols), global_count=global_batch) if wl["train"]
              else Inference(model))

    graphed = False
    if not args.eager:
        runner.capture(batch)  # its warm-up steps are extra, untimed
        graphed = True
    for _ in range(args.warmup):
        runner.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = runner.step(batch)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t.item())
    final_loss = float(loss.item())

    if args.step_only:
        if rank == 0:
            print(json.dumps({"value": round(global_batch * args.steps / t_max, 2),
                              "ms_per_step": round(1e3 * t_max / args.steps, 4), "steps": args.steps,
                              "final_loss": float(f"{final_loss:.6e}")}),
                  flush=True)
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return

    meta = batch.host_meta()
    traffic_path, traffic_table = load_traffic(args.workload, args.shape)
    probe, shape = attention_probe(model, batch, args.kernel_reps, train=wl["train"])
    plan_lg = model.line_graph_data(batch)[1].lg
    sa = scatter_add_probe(plan_lg, args.kernel_reps)
    dense = dense_probe(shape["E"], args.kernel_reps)
    dense.update(chain_probe(shape["E"], args.kernel_reps))
    if wl["train"]:
        dense.update(proj_probe(shape["E"], args.kernel_reps))
    # the roofline kernel: the step's largest single kernel in the committed profile
    # (profiles/r2_*_step_kernels.txt) -- the one-launch T-layout weight gradient of the whole
    # backward (x2g_tiled_wgrad_flat), f32 MFMA-bound (sum_j 2 R 128 cols_j FLOP, ~K = R deep)
    roof = None
    flat = flat_wgrad_probe(runner.flat_launches, args.kernel_reps) if wl["train"] else None
    if flat is not None:
        # the launch's duration inside the step (eager passes, HIP events around it on its stream): the
        # roofline figure; the probe (the same launch back to back on synthetic operands that are not
        # MALL-resident) beside it
        in_ms, in_n = in_step_kernel_ms(runner, batch, "tiled_wgrad_flat", max(3, args.kernel_reps // 4))
        f_ms = in_ms if in_ms is not None else flat["ms"]
        f_tfs = flat["flops"] / (f_ms * 1e-3) / 1e12
        p_tfs = flat["flops"] / (flat["ms"] * 1e-3) / 1e12
        traffic = pmc_traffic([("tiled_flat_kernel", None)], traffic_table)  # (the largest launch)
        roof = {"kernel": f"x2g_tiled_wgrad_flat: {flat['jobs']} weight gradients dW = dz^T x over "
                          f"R={flat['rows']} rows in one launch (tiled_flat_kernel)",
                "bound": "mfma", "achieved": round(f_tfs, 2), "peak": MFMA_F32_PEAK_TFS,
                "unit": "TFLOP/s", "frac": round(f_tfs / MFMA_F32_PEAK_TFS, 4), "traffic": traffic,
                "avg_ms": round(f_ms, 5), "timing": (f"in-step: median of {in_n} eager training passes, HIP "
                                                     f"events around the launch on its stream" if in_ms is not None
                                                     else "probe"),
                "probe_ms": round(flat["ms"], 5), "probe_frac": round(p_tfs / MFMA_F32_PEAK_TFS, 4),
                "flops_per_launch": int(flat["flops"]),
                "traffic_source": os.path.relpath(traffic_path, ROOT) if traffic else None}
        dense["tiled_wgrad_flat"] = (f_ms, flat["flops"])
    if not wl["train"]:  # inference: no backward; the T-row attention forward dominates
        a_ms, a_bytes, a_gath = probe["attn_fwd"]
        a_gbs = a_bytes / (a_ms * 1e-3) / 1e9
        hbm = _pmc_bytes("attn_fwd", traffic_table)
        roof = {"kernel": ("x2g_sbf_attention_fwd_center_sf_tiled + _sf (attn_fwd_center_sf_tiled_kernel / "
                           "attn_fwd_center_sf_kernel: lin_sbf fused, one workgroup per center atom (sources in tiles "
                           "of 16 for degrees > 17) or per pack of small atoms; no S = lin_sbf(sbf) exists)"
                           if shape.get("sf") else
                           "x2g_sbf_attention_fwd_center (attn_fwd_center_kernel: one workgroup per center atom, "
                           "S = lin_sbf(sbf) precomputed)" if shape.get("center") else
                           "x2g_sbf_attention_fwd (attn_fwd_batched, S = lin_sbf(sbf) precomputed)"),
                "bound": "hbm", "achieved": round(a_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(a_gbs / HBM_PEAK_GBS, 4), "traffic": hbm, "avg_ms": round(a_ms, 5),
                "bytes_per_launch": int(a_bytes), "gathered_bytes_per_launch": int(a_gath),
                "hbm_GBs": None if hbm is None else round(hbm / (a_ms * 1e-3) / 1e9, 1),
                "traffic_source": os.path.relpath(traffic_path, ROOT) if hbm is not None else None}
    if args.workload == "aid_infer":
        data_desc = (f"AID_kcal geometries (tests/golden/aid_geom.npz = the reference's raw/AID_kcal.xyz; "
                     f"{meta['nodes'].mean():.1f} atoms, {meta['edges'].mean():.0f} directed edges, "
                     f"{meta['triplets'].mean():.0f} triplets per molecule), random 338-wide edge features, "
                     f"random-init weights")
        work = "xgnn_poly U0 inference (config.json widths), forward only, energies"
    else:
        data_desc = (f"synthetic QM9-shaped molecules ({args.shape}: ~18 atoms, {meta['edges'].mean():.0f} "
                     f"directed edges, {meta['triplets'].mean():.0f} triplets per molecule, random 338-wide "
                     f"edge features), random-init weights")
        kind = "xgnn_poly U0" if args.workload == "qm9_u0" else (
            f"target {args.target} ({LABELS[args.target]}) "
            f"{'xgnn_poly AtomWise' if global_pool is None else 'xgnn_poly_global MolWise mean-pool'}")
        work = (f"{kind} train step (config.json: L=4, D=128, H=16, sbf 7x6), {args.shape}, "
                f"fwd+loss+bwd+allreduce+clip+Adam+EMA")

    if rank == 0:
        line = {
            "metric": wl["metric"],
            "value": round(global_batch * args.steps / t_max, 2),
            "unit": "molecules/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * t_max / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": data_desc,
            "config": {"workload": work,
                       "per_gpu_batch": len(mols), "global_batch": global_batch,
                       "sharding": "one global batch, shard_by_triplets (sum-T balanced)" if world > 1 else None,
                       "shard_triplets": shard_t if world > 1 else None,
                       "imbalance_max_over_mean": (round(max(shard_t) / (sum(shard_t) / world), 5)
                                                   if world > 1 else None),
                       "line_nodes_per_gpu": shape["E"], "triplets_per_gpu": shape["T"],
                       "parallelism": f"dp{world}", "hip_graph": graphed,
                       "grad_allreduce": None if world == 1 else (
                           "RCCL" if args.dist_backend == "nccl" else "gloo (rehearsal)")},
            "roofline": roof,
            "step_roofline": step_roofline(round(1e3 * t_max / args.steps, 4), args.workload, args.shape),
            "kernels": dict(
                {k: _hbm_entry(k, v, traffic_table) for k, v in probe.items()},
                **{k: _mfma_entry(k, v, traffic_table) for k, v in dense.items()}),
            "roofline_scatter_add": {
                "kernel": "x2g_segment_sum [T,128]->[E,128]", "bytes_per_launch": sa["bytes"],
                "warm_GBs": round(sa["bytes"] / (sa["warm_ms"] * 1e-3) / 1e9, 1),
                "cold_GBs": round(sa["bytes"] / (sa["cold_ms"] * 1e-3) / 1e9, 1),
                "cold_frac": round(sa["bytes"] / (sa["cold_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "parity": sa["parity"]},
            ("final_loss" if wl["train"] else "energy_sum"): float(f"{final_loss:.6e}"),  # (one resident batch: memorised)
            # per-batch host cost a loader must hide under the step (not in `value`: inputs are
            # resident in HBM when the timed region starts)
            "host_batch_ms": {"collate": round(1e3 * (t_c1 - t_c0), 3), "h2d": round(1e3 * (t_c2 - t_c1), 3),
                              "molecules": len(mols)},
        }
        if wl["train"] and world == 1 and args.workload == "qm9_u0" and not args.no_loader:
            line["loader"] = loader_probe(CFG, dev, shape=args.shape)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(mols, args.cpu_seconds, global_pool=global_pool, train=wl["train"],
                                                sample=8 if args.workload == "aid_infer" else None)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
