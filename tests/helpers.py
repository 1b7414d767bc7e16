"""Test helpers: rebuild fixture inputs as batches, seeded models, comparisons."""
import numpy as np
import torch

from conftest import golden  # noqa: F401
from weights import load_seeded


def batch_from_fixture(z, prefix="", shipped=True):
    """Collated x2gnn Batch (host) from a fixture's stored inputs.  ``shipped``: with the index forms
    collate attaches (symmetric flag, largest degree, center order / packs / atom_info, per-molecule
    triplet counts), so a model runs the path a training batch takes (the center-atom attention kernels
    at D = 128); False: the bare tensors, which take the generic line-graph build and the
    destination-major attention kernels."""
    from x2gnn.data import Batch, Data, _add_device_indices

    nodes, edges, trips = z[prefix + "nodes"], z[prefix + "edges"], z[prefix + "triplets"]
    b = Batch()
    b._store["x"] = torch.from_numpy(z[prefix + "x"].astype(np.int64))
    b._store["atom_pos"] = torch.from_numpy(z[prefix + "atom_pos"])
    b._store["edge_index"] = torch.from_numpy(z[prefix + "edge_index"].astype(np.int64))
    b._store["edge_attr"] = torch.from_numpy(z[prefix + "edge_attr"])
    b._store["edge_num"] = torch.from_numpy(edges.astype(np.int64))
    b._store["y"] = torch.from_numpy(z[prefix + "y"])
    b._store["batch"] = torch.repeat_interleave(torch.arange(len(nodes)), torch.from_numpy(nodes.astype(np.int64)))
    b._store["ptr"] = torch.from_numpy(np.concatenate([[0], np.cumsum(nodes)]).astype(np.int64))
    object.__setattr__(b, "_meta", {"nodes": nodes.astype(np.int64), "edges": edges.astype(np.int64),
                                    "triplets": trips.astype(np.int64)})
    if shipped:
        _add_device_indices(b, nodes.astype(np.int64), edges.astype(np.int64))
    assert isinstance(b, Data)
    return b


def model_cfg(z):
    return dict(zip([str(k) for k in z["cfg_keys"]], [int(v) for v in z["cfg_vals"]]))


def pool_option(z):
    return str(z["pool_option"]) if "pool_option" in z.files else "mean"


def oracle_model(z):
    from oracle.ref_cpu import XGNN

    kind = str(z["kind"])
    m = XGNN(global_pool=pool_option(z) if kind == "global" else None, **model_cfg(z))
    load_seeded(m, int(z["weight_seed"]))
    return m


def rel_err(a, b):
    """max |a - b| / max |b| (one scale for the whole array: outputs other than energies)."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def energy_rel_err(a, b, floor=1e-3):
    """Per-molecule relative error of energies: max_i |a_i - b_i| / |b_i| — the north-star "1e-4
    relative on fp32 energies" per molecule, not against the batch maximum.  A molecule whose
    reference energy is below ``floor`` x the batch's largest magnitude is measured against that
    floor instead (a relative error of a near-zero value is not meaningful)."""
    a = np.asarray(a, np.float64).reshape(-1)
    b = np.asarray(b, np.float64).reshape(-1)
    if b.size == 0:
        return 0.0
    scale = np.maximum(np.abs(b), floor * max(np.abs(b).max(), 1e-30))
    return float((np.abs(a - b) / scale).max())
