"""Work partition across GPUs (one process per GPU, torch.distributed launch).

The reference's only parallelism is 8 row bands over std::threads (src/main.cpp:38-39,
164-185).  Pixels and samples have no cross-dependency, so ranks split work with no
collective on the data path:

* ``sample_range``: sample-parallel -- rank r takes a contiguous block of the camera's
  samples (the accumulation buffers (sum w*c, sum w) add across ranks; the host resolves);
* ``row_band``: row bands like main.cpp:38-39, but covering every row (the reference
  drops the H % 8 remainder rows: a quirk not reproduced for N ranks);
* ``gather_rows``: host-side gather of row bands into one framebuffer.

Results are independent of the number of ranks: the counter-based RNG is keyed by
(pixel, sample, ray-tree node), not by thread or device.
"""
from __future__ import annotations

import numpy as np


def sample_range(rank: int, world: int, spp: int):
    """Contiguous samples [begin, begin+count) of rank ``rank`` among ``world``."""
    base, extra = divmod(spp, world)
    begin = rank * base + min(rank, extra)
    return begin, base + (1 if rank < extra else 0)


def row_band(rank: int, world: int, height: int):
    """Rows [y0, y1) of rank ``rank``; the last band takes the remainder."""
    step = height // world
    y0 = rank * step
    y1 = height if rank == world - 1 else y0 + step
    return y0, y1


def gather_rows(bands, height: int, width: int, channels: int = 3, dtype=np.float32):
    """bands: iterable of ((y0, y1), rows_array[y1-y0, width, channels])."""
    out = np.zeros((height, width, channels), dtype)
    for (y0, y1), a in bands:
        out[y0:y1] = a
    return out
