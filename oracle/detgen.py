"""Deterministic, counter-based data/weight generator (TEST INFRASTRUCTURE).

Every tensor used by the parity tests is a pure function of (seed, name, shape):
splitmix64 over a counter, so the same bytes come out in this container, on the
GPU box, and in any numpy version.  This lets the 53.6 MB Stage-4 weight set be
regenerated instead of committed (SURVEY.md §8c "Determinism recipe").
"""
from __future__ import annotations

import numpy as np
import torch

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def _fnv1a64(s: str) -> int:
    h = 0xCBF29CE484222325
    for b in s.encode():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def stream_seed(seed: int, name: str = "") -> int:
    return (_fnv1a64(name) ^ (int(seed) * 0x9E3779B97F4A7C15)) & 0xFFFFFFFFFFFFFFFF


def uniform(seed: int, n: int, name: str = "") -> np.ndarray:
    """n float64 samples in [0, 1)."""
    base = np.uint64(stream_seed(seed, name))
    with np.errstate(over="ignore"):
        ctr = (np.arange(n, dtype=np.uint64) * np.uint64(0xD1B54A32D192ED03) + base) & _M64
    bits = _splitmix64(ctr) >> np.uint64(11)
    return bits.astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed: int, n: int, name: str = "") -> np.ndarray:
    m = (n + 1) // 2
    u1 = uniform(seed, m, name + "#bm1")
    u2 = uniform(seed, m, name + "#bm2")
    r = np.sqrt(-2.0 * np.log(1.0 - u1))
    out = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])
    return out[:n]


def randn(seed: int, shape, name: str = "", dtype=torch.float32) -> torch.Tensor:
    n = int(np.prod(shape))
    return torch.from_numpy(normal(seed, n, name).reshape(shape)).to(dtype)


def bernoulli(seed: int, shape, p: float = 0.5, name: str = "") -> torch.Tensor:
    n = int(np.prod(shape))
    return torch.from_numpy((uniform(seed, n, name) < p).astype(np.float32).reshape(shape))


def randint(seed: int, shape, high: int, name: str = "") -> torch.Tensor:
    n = int(np.prod(shape))
    return torch.from_numpy(np.floor(uniform(seed, n, name) * high).astype(np.int64).reshape(shape))


def init_tensor(seed: int, name: str, shape) -> torch.Tensor:
    """Deterministic value for one state_dict entry, chosen by its key name.

    Conv/Linear weights and biases: U(-1/sqrt(fan_in), +1/sqrt(fan_in)) (the
    bound PyTorch's default init uses).  BatchNorm affine/running stats are set
    away from their identity defaults so the tests exercise every term.
    """
    shape = tuple(shape)
    n = int(np.prod(shape)) if len(shape) else 1
    leaf = name.rsplit(".", 1)[-1]
    u = uniform(seed, n, name)
    if leaf == "num_batches_tracked":
        return torch.tensor(0, dtype=torch.int64)
    if leaf == "running_mean":
        v = 0.2 * (2 * u - 1)
    elif leaf == "running_var":
        v = 0.5 + u
    elif len(shape) == 1 and _is_bn_param(name):
        v = (1.0 + 0.5 * (2 * u - 1)) if leaf == "weight" else 0.2 * (2 * u - 1)
    else:
        fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else None
        if fan_in is None:  # a bias: use the fan-in of its weight, passed via name lookup
            fan_in = _BIAS_FAN_IN.get(name, shape[0])
        b = 1.0 / np.sqrt(fan_in)
        v = b * (2 * u - 1)
    return torch.from_numpy(v.reshape(shape)).to(torch.float32)


_BIAS_FAN_IN: dict = {}
_BN_NAMES: set = set()


def _is_bn_param(name: str) -> bool:
    return name.rsplit(".", 1)[0] in _BN_NAMES


def make_state(spec, seed: int) -> dict:
    """spec: ordered list of (name, shape, kind) with kind in {conv, linear, bn, bias}."""
    # record bias fan-ins and BN module prefixes for init_tensor
    shapes = {n: s for n, s, _ in spec}
    for n, s, kind in spec:
        if kind == "bn":
            _BN_NAMES.add(n.rsplit(".", 1)[0])
    for n, s, kind in spec:
        if n.endswith(".bias") and kind != "bn":
            w = n[: -len("bias")] + "weight"
            if w in shapes:
                _BIAS_FAN_IN[n] = int(np.prod(shapes[w][1:]))
    return {n: init_tensor(seed, n, s) for n, s, _ in spec}
