"""Deterministic parameter values for parity fixtures (test infrastructure).

The reference's checkpoints are missing (.MISSING_LARGE_BLOBS), so fixtures use seeded random
weights.  Rather than committing megabytes of weights, every tensor is drawn from numpy's
PCG64 seeded by (seed, crc32(parameter name)) — reproducible on any machine — and the same
function loads them into the reference (fixture generation) and into this framework (tests).
"""
from __future__ import annotations

import math
import zlib

import numpy as np
import torch


def seeded_value(name: str, shape, seed: int) -> np.ndarray:
    rng = np.random.default_rng([seed, zlib.crc32(name.encode())])
    shape = tuple(shape)
    if name.endswith("frequencies"):
        return (math.pi * np.arange(1, shape[0] + 1) + 0.05 * rng.standard_normal(shape)).astype(np.float32)
    if name.endswith("embedding.weight"):
        w = rng.standard_normal(shape).astype(np.float32)
        w[0] = 0.0  # padding row
        return w
    if len(shape) == 1:
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    fan_out, fan_in = shape[0], int(np.prod(shape[1:]))
    return (rng.standard_normal(shape) * math.sqrt(2.0 / (fan_in + fan_out))).astype(np.float32)


def load_seeded(module: torch.nn.Module, seed: int) -> dict:
    """Overwrite every parameter of ``module`` in place; returns {name: numpy value}."""
    vals = {}
    with torch.no_grad():
        for name, p in module.named_parameters():
            v = seeded_value(name, p.shape, seed)
            p.copy_(torch.from_numpy(v))
            vals[name] = v
    return vals
