"""TEST INFRASTRUCTURE ONLY -- deterministic, name-keyed value filler.

Weights and inputs for every parity case are generated from (name, flat index)
by SplitMix64, so that the golden-vector generator (which imports the
reference, in the build container only), the CPU oracle and the GPU tests all
see bit-identical fp32 tensors without committing multi-GB weight files
("Golden-vector plan").

value(name, i) = offset + scale * (2 * u - 1),   u = (splitmix64(crc32(name) << 32 ^ i) >> 40) / 2**24

u has 24 random bits, so 2u-1 is exact in fp32 and the result is one fp32
rounding of offset + scale * (2u - 1).
"""
from __future__ import annotations

import zlib

import numpy as np

_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def uniform_bits(name: str, n: int, start: int = 0) -> np.ndarray:
    """24-bit uniforms in [0, 1) as float64 for flat indices [start, start+n)."""
    key = np.uint64(zlib.crc32(name.encode("utf-8")) & 0xFFFFFFFF) << np.uint64(32)
    idx = np.arange(start, start + n, dtype=np.uint64)
    z = _splitmix64(key ^ idx)
    return (z >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)


def fill(name: str, shape, scale: float = 1.0, offset: float = 0.0,
         chunk: int = 1 << 24) -> np.ndarray:
    """fp32 array of `shape` with values offset + scale*U(-1,1), keyed by `name`."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    out = np.empty(n, dtype=np.float32)
    for s in range(0, n, chunk):
        m = min(chunk, n - s)
        u = uniform_bits(name, m, s)
        out[s:s + m] = (offset + scale * (2.0 * u - 1.0)).astype(np.float32)
    return out.reshape(shape)


def randint(name: str, shape, low: int, high: int) -> np.ndarray:
    """int64 array uniform in [low, high), keyed by `name`."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    u = uniform_bits(name, n)
    v = low + np.floor(u * (high - low)).astype(np.int64)
    return np.minimum(v, high - 1).reshape(shape)


def bernoulli(name: str, shape, p: float) -> np.ndarray:
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    return (uniform_bits(name, n) < p).astype(np.int32).reshape(shape)


def param_spec(name: str, shape) -> tuple[float, float]:
    """(scale, offset) used for a reference state_dict key in parity cases.

    Chosen so activations stay O(1) and LayerNorm outputs have row sums far
    from zero (beta random), which keeps the reference's exact-zero key/query
    masks (modules.py:257, :289) deterministic across summation orders.
    """
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "gamma":
        return 0.2, 1.0
    if leaf == "beta":
        return 0.2, 0.0
    if name.endswith("syb_emb.weight"):
        return 0.5, 0.0
    if leaf == "lookup_table":
        if ".dec_emb." in "." + name:
            return 0.05, 0.0
        return 0.5, 0.0
    if leaf in ("weight", "bias"):
        # nn.Linear: fan_in is the last dim of the weight (bias: caller passes fan_in via shape hint)
        fan_in = shape[-1] if leaf == "weight" and len(shape) >= 2 else None
        if fan_in is None:
            return 0.02, 0.0
        return 1.0 / float(np.sqrt(fan_in)), 0.0
    return 0.02, 0.0


def param_value(name: str, shape) -> np.ndarray:
    scale, offset = param_spec(name, shape)
    return fill("param:" + name, shape, scale, offset)


class HashParams(dict):
    """Lazy name -> fp32 torch tensor map of hash-filled reference parameters."""

    def __init__(self, requires_grad=False, num_relations=4, **geometry):
        super().__init__()
        self.requires_grad = requires_grad
        from .savqa_oracle import model_param_shapes
        self.shapes = dict(model_param_shapes(num_relations=num_relations, **geometry))

    def __missing__(self, name):
        import torch
        shape = self.shapes[name] if name in self.shapes else None
        if shape is None:
            raise KeyError(name)
        t = torch.from_numpy(param_value(name, shape)).requires_grad_(self.requires_grad)
        self[name] = t
        return t
