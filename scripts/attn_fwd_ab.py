"""Attention forward at config 2: S = lin_sbf(sbf) precomputed (x2g_sbf_project + the batched
PRE kernel, the default) vs the projection computed on the fly inside the attention kernel
(w_sbf passed: attn_fwd_kernel<PRE=false>).  Interleaved, minimum over rounds."""
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "x2-gnn_amd"))
import bench  # noqa: E402
import x2gnn  # noqa: E402
from x2gnn import ops  # noqa: E402
from x2gnn._lib import call, ptr, stream_ptr  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.synth import synthetic_molecules  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
model = x2gnn.xgnn_poly(device="cuda", **bench.CFG).to(dev)
batch = collate(synthetic_molecules(128, "S160", seed=1000)).to(dev)
conv = model.fin_model.convs[0]
line, plan = model.line_graph_data(batch)
lg = plan.lg
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
f32 = dict(dtype=torch.float32, device=dev)
out1, out2 = torch.empty(E, D, **f32), torch.empty(E, D, **f32)
alpha, smax, sden = torch.empty(T, H, **f32), torch.empty(E, H, **f32), torch.empty(E, H, **f32)
sproj = torch.empty(T, D, **f32)
S = sbf.shape[1]


def pre():
    call("x2g_sbf_project", ptr(sbf), T, S, ptr(W), ptr(bsb), D, ptr(sproj), stream_ptr())
    call("x2g_sbf_attention_fwd", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(row), ops.EDGE_PER_DST,
         ptr(sproj), None, None, ptr(lg.trip_rowptr), ptr(lg.trip_src), E, T, H, C, D, ptr(out1), ptr(alpha),
         ptr(smax), ptr(sden), stream_ptr())


def onfly():
    call("x2g_sbf_attention_fwd", ptr(q), ptr(k), ptr(v), ptr(skip), ptr(table), ptr(row), ops.EDGE_PER_DST,
         ptr(sbf), ptr(W), ptr(bsb), ptr(lg.trip_rowptr), ptr(lg.trip_src), E, T, H, C, S, ptr(out2), ptr(alpha),
         ptr(smax), ptr(sden), stream_ptr())


def t(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


pre()
onfly()
torch.cuda.synchronize()
print("max |out diff|", float((out1 - out2).abs().max()), flush=True)
best = {}
for rnd in range(4):
    for name, fn in ((("pre", pre), ("onfly", onfly)) if rnd % 2 == 0 else (("onfly", onfly), ("pre", pre))):
        best[name] = min(best.get(name, 1e9), t(fn))
print(f"projection + batched PRE attention: {best['pre']:.1f} us; on-the-fly attention: {best['onfly']:.1f} us",
      flush=True)
