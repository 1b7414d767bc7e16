"""Training-trajectory check of the bench's step (GPU): the smooth-L1 loss over N steps on the bench's
own batch for (a) x2gnn.train.Trainer replayed from its captured HIP graphs, (b) the same Trainer
eager, and (c) the reference trainer's step written with plain torch (model forward, F.smooth_l1_loss,
loss.backward(), clip_grad_norm_(100), torch.optim.Adam(1e-3), trainer.py:37-48) on the same model
code.  The three trajectories must agree to fp32 reassociation drift.

    python scripts/loss_check.py [steps] [batch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "x2-gnn_amd")]

import torch  # noqa: E402

import x2gnn  # noqa: E402
from x2gnn.data import collate  # noqa: E402
from x2gnn.synth import synthetic_molecules  # noqa: E402
from x2gnn.train import Trainer  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 225
B = int(sys.argv[2]) if len(sys.argv) > 2 else 128
CFG = dict(conv_layers=4, sbf_dim=7, rbf_dim=6, in_channels=128, heads=16, embedding_size=128)
dev = torch.device("cuda", 0)
batch = collate(synthetic_molecules(B, "S160", seed=1000)).to(dev)
marks = sorted({0, 1, 2, 5, 10, 25, 50, 100, steps - 1} & set(range(steps)))


def fresh():
    torch.manual_seed(0)
    return x2gnn.xgnn_poly(device="cuda", **CFG).to(dev)


def run_trainer(graphed):
    tr = Trainer(fresh())
    if graphed:
        tr.capture(batch, warm=1)
    out = {}
    for i in range(steps):
        loss = tr.step(batch)
        if i in marks:
            out[i] = float(loss)
    return out


def run_torch():
    m = fresh()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    out = {}
    for i in range(steps):
        opt.zero_grad(set_to_none=True)
        loss = torch.nn.functional.smooth_l1_loss(m(batch), batch.y)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(m.parameters(), 100.0)
        opt.step()
        if i in marks:
            out[i] = float(loss)
    return out


res = {"trainer_graph": run_trainer(True), "trainer_eager": run_trainer(False), "torch_autograd": run_torch()}
print(f"batch {B}, y mean {float(batch.y.mean()):.4f} std {float(batch.y.std()):.4f}")
print("step  " + "  ".join(f"{k:>16s}" for k in res))
for i in marks:
    print(f"{i:4d}  " + "  ".join(f"{res[k][i]:16.8f}" for k in res))
