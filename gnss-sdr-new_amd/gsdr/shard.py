"""Multi-GPU sharding of the acquisition + tracking path.

One process per GPU.  The work units are independent, so they are partitioned
with no data-path collective:

* acquisition: consecutive 1 ms blocks of the IQ stream (every block is a full
  PRN x Doppler grid, pcps_acquisition.cc:615-882, with no state carried from one
  block to the next in single-dwell mode) -- rank r owns the contiguous block
  range ``block_range(total, world, r)``;
* tracking: channels (each dll_pll_veml_tracking instance is a serial loop over
  its own epochs, dll_pll_veml_tracking.cc:1784-2152) -- channel c lives on rank
  ``c % world``, a fixed map (unlike the reference CUDA path's
  ``rand() % num_devices``, cuda_multicorrelator.cu:150-154).

The only cross-rank traffic is the result merge on the host (results are small:
one record per (block, PRN) and per channel epoch) and the benchmark's barrier /
max-over-ranks timing.  ``merge_*`` restore the single-process order.
"""
import numpy as np


def block_range(total_blocks, world, rank):
    """Contiguous block span [lo, hi) of rank `rank`; the first total % world ranks
    take one extra block."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank %r/%r" % (world, rank))
    q, r = divmod(int(total_blocks), world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def channels_of(n_channels, world, rank):
    """Channel ids tracked on `rank` (fixed map c % world)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank %r/%r" % (world, rank))
    return np.arange(rank, int(n_channels), world, dtype=np.int64)


def merge_blocks(per_rank, total_blocks, world):
    """Concatenate per-rank acquisition results (each rank's array is its block
    span, block-major) back into stream order; checks the spans tile the stream."""
    out = []
    for r in range(world):
        lo, hi = block_range(total_blocks, world, r)
        part = per_rank[r]
        if len(part) != hi - lo:
            raise ValueError("rank %d returned %d blocks, owns %d" % (r, len(part), hi - lo))
        out.append(part)
    return np.concatenate(out) if out else np.empty(0)


def merge_channels(per_rank, n_channels, world):
    """Per-channel records from every rank, indexed by global channel id."""
    merged = [None] * int(n_channels)
    for r in range(world):
        ids = channels_of(n_channels, world, r)
        if len(per_rank[r]) != len(ids):
            raise ValueError("rank %d returned %d channels, owns %d" % (r, len(per_rank[r]), len(ids)))
        for c, rec in zip(ids, per_rank[r]):
            merged[int(c)] = rec
    return merged
