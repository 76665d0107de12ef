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
