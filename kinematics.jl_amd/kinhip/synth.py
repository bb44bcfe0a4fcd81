"""Synthetic joint configurations: a counter-based hash of
(seed, global configuration index, column), so that every rank of a sharded
run generates exactly its slice of one global dataset with no scatter.
"""
from __future__ import annotations

import math

import torch

_M64 = (1 << 64) - 1


def _s64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


_GOLD = _s64(0x9E3779B97F4A7C15)
_C1 = _s64(0xBF58476D1CE4E5B9)
_C2 = _s64(0x94D049BB133111EB)


def _srl(x: torch.Tensor, k: int) -> torch.Tensor:  # logical shift right on int64
    return (x >> k) & ((1 << (64 - k)) - 1)


def splitmix64(x: torch.Tensor) -> torch.Tensor:
    z = x + _GOLD
    z = (z ^ _srl(z, 30)) * _C1
    z = (z ^ _srl(z, 27)) * _C2
    return z ^ _srl(z, 31)


def uniform_configs(lower, upper, n: int, start: int = 0, seed: int = 20261015, dtype=torch.float32,
                    device=None) -> torch.Tensor:
    """(len(lower), n) tensor, column c ~ U[lower[c], upper[c]] (U[-pi, pi] where a
    limit is infinite), for global configuration indices [start, start + n)."""
    ncol = len(lower)
    idx = torch.arange(start, start + n, dtype=torch.int64, device=device)
    out = torch.empty((ncol, n), dtype=torch.float64, device=device)
    for c in range(ncol):
        lo, hi = float(lower[c]), float(upper[c])
        if not (math.isfinite(lo) and math.isfinite(hi)):
            lo, hi = -math.pi, math.pi
        key = idx * ncol + c
        z = splitmix64(key * _GOLD + _s64(seed))
        u = _srl(z, 11).to(torch.float64) * (1.0 / (1 << 53))
        out[c] = lo + (hi - lo) * u
    return out.to(dtype)
