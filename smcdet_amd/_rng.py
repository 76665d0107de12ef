"""Counter-based random streams for the HIP kernels.

Every kernel draws from Philox4x32-10 keyed by a 64-bit seed, with a 64-bit
counter base ("offset") that the host advances by the number of counters a
launch consumes.  The seed is taken from torch's default CPU generator, so
`torch.manual_seed(s)` makes a whole run reproducible, as it does for the
reference (whose draws come from torch.rand / Tensor.multinomial).
"""
from __future__ import annotations

import torch


def torch_seed() -> int:
    """A 63-bit seed drawn from torch's default CPU generator."""
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


def rank_seed(seed, rank: int) -> int:
    """Seed of rank `rank`'s streams in a sharded run.  The kernels key their
    draws by the rank-local tile/particle index, so ranks must not share a
    seed (under torchrun every rank's torch.manual_seed is usually the same).
    Rank 0 keeps the base seed, so a one-rank shard reproduces the
    single-process sampler with that seed; other ranks get a splitmix64 mix
    of (base, rank).  seed None: the base comes from torch's generator."""
    base = torch_seed() if seed is None else int(seed) & ((1 << 64) - 1)
    if rank == 0:
        return base
    z = (base + 0x9E3779B97F4A7C15 * (rank + 1)) & ((1 << 64) - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return (z ^ (z >> 31)) & ((1 << 63) - 1)


class PhiloxStream:
    def __init__(self, seed: int | None = None):
        self.seed = torch_seed() if seed is None else int(seed) & ((1 << 64) - 1)
        self.offset = 0

    def take(self, n: int) -> int:
        """Reserves n counters; returns the base offset of the block."""
        base = self.offset
        self.offset += max(int(n), 1)
        return base

    def state(self):
        return {"seed": self.seed, "offset": self.offset}

    def load_state(self, st):
        self.seed = int(st["seed"])
        self.offset = int(st["offset"])
