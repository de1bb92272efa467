"""ttdist — multi-GPU sharding of the trace path (one process per GPU).

The reference is single-GPU. On an 8×MI355X node the scene is replicated per GPU (it is at most
~1.5 GB) and the rays are sharded; rays never interact, so the only collective is an optional
gather of the 16-byte hit records to rank 0 (RCCL via torch.distributed "nccl", or "gloo" on
CPU in the tests).

Three shardings:
  * ``spp`` (weak scaling, bench.py default at N > 1): the job at N ranks is an N-sample 1080p frame
    (sample k = the reference's Generate with frames_accumulated = k); its (sample, 64x64 tile) units
    are dealt round-robin to the ranks (``spp_part_pixels``), so every rank traces one frame's worth of
    screen tiles -- the north star's tile sharding at fixed per-GPU work -- and the primary hit records
    of all N samples are gathered to rank 0 (``assemble_spp``).
  * ``tiles`` (strong scaling, SURVEY.md §8(e), ``bench.py --shard tiles``): the screen is cut into
    ``tile``×``tile`` pixel tiles dealt round-robin to ranks (balances sky-heavy and geometry-heavy
    regions); each rank builds a compact ray list of its pixels (optionally split into
    tile-interleaved parts, ``part_pixels``) and the hit records are gathered and scattered back
    into screen order on rank 0.
  * ``sample`` (weak scaling, ``bench.py --shard sample`` and the ``aux_sample_sharded`` line):
    every rank traces its own full-frame sample of the same view (``frames_accumulated = rank``
    selects the sub-pixel jitter).
"""
from __future__ import annotations

from typing import List

import numpy as np


def lpt_owner(costs, world: int) -> np.ndarray:
    """Longest-processing-time-first deal of tiles to ranks: tiles in descending cost (ties: lower tile
    id first), each to the rank with the least cost so far (ties: lower rank). Deterministic, so every
    rank computes the same deal from the same costs. Returns owner[tile]."""
    costs = np.asarray(costs, np.float64)
    order = np.lexsort((np.arange(len(costs)), -costs))
    loads = np.zeros(world, np.float64)
    owner = np.zeros(len(costs), np.int64)
    for t in order:
        r = int(np.argmin(loads))
        owner[t] = r
        loads[r] += costs[t]
    return owner


def tile_costs_from_chunks(chunk_costs, width: int, height: int, tile: int = 64, floor: int = 24) -> np.ndarray:
    """Per-tile cost of a full-frame launch from its 8x8-chunk cost map (tthip.Engine.chunk_costs, bounce 0
    with TT_TRACE_ADAPTIVE_ORDER): the sum over the tile's chunks of max(chunk cost, floor) -- the map
    records a chunk's largest Reps count only when it reaches 32 node steps, so `floor` stands for the
    cheap chunks (C2's mean is ~16 node steps per ray)."""
    cw, ch = width // 8, height // 8
    cm = np.maximum(np.asarray(chunk_costs, np.float64)[: cw * ch].reshape(ch, cw), floor)
    tx, ty = (width + tile - 1) // tile, (height + tile - 1) // tile
    k = tile // 8
    out = np.zeros(tx * ty, np.float64)
    for t in range(tx * ty):
        x0, y0 = (t % tx) * k, (t // tx) * k
        out[t] = cm[y0:y0 + k, x0:x0 + k].sum()
    return out


def _rank_tiles(n_t: int, world: int, rank: int, owner=None):
    return range(rank, n_t, world) if owner is None else [int(t) for t in np.nonzero(np.asarray(owner) == rank)[0]]


def virtual_owner(owner, world: int, parts: int) -> np.ndarray:
    """A deal of tiles to ranks, with each rank's tiles split into ``parts`` interleaved parts: part s of
    rank r is virtual rank s * world + r (its tiles in increasing id, every parts-th one), as part_pixels."""
    owner = np.asarray(owner)
    out = np.zeros_like(owner)
    for r in range(world):
        for i, t in enumerate(np.nonzero(owner == r)[0]):
            out[t] = (i % parts) * world + r
    return out


def tile_pixels(width: int, height: int, world: int, rank: int, tile: int = 64, block: int = 8,
                owner=None) -> np.ndarray:
    """Pixel indices owned by ``rank`` in tile order: round-robin tile sharding (tile t to rank t % world), or
    the deal ``owner[t]`` (lpt_owner). Inside a tile the pixels run in ``block``x``block`` sub-blocks
    (row-major blocks, row-major pixels in a block), so the 64 rays a wave dequeues together are an 8x8
    screen patch, as the trace kernel's own swizzle makes them for full-frame batches."""
    tx, ty = (width + tile - 1) // tile, (height + tile - 1) // tile
    out = []
    for t in _rank_tiles(tx * ty, world, rank, owner):
        x0, y0 = (t % tx) * tile, (t // tx) * tile
        ys, xs = np.meshgrid(np.arange(y0, min(y0 + tile, height)), np.arange(x0, min(x0 + tile, width)),
                             indexing="ij")
        ys, xs = ys.reshape(-1), xs.reshape(-1)
        order = np.lexsort((xs, ys, (xs - x0) // block, (ys - y0) // block))
        out.append((ys * width + xs)[order])
    return np.concatenate(out).astype(np.int64) if out else np.zeros(0, np.int64)


def shard_sizes(width: int, height: int, world: int, tile: int = 64, owner=None) -> List[int]:
    return [len(tile_pixels(width, height, world, r, tile, owner=owner)) for r in range(world)]


def gather_hits(hits, world: int, rank: int, dst: int = 0):
    """Gathers each rank's (n_r, 4) uint32/int32 hit-record tensor to ``dst``. Shards may differ
    in length, so they are padded to the largest shard (one collective, equal message sizes).
    Returns the list of per-rank tensors on ``dst`` (trimmed), None elsewhere."""
    import torch
    import torch.distributed as dist

    n = torch.tensor([hits.shape[0]], dtype=torch.int64, device=hits.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s.item()) for s in sizes))
    pad = torch.zeros((m, hits.shape[1]), dtype=hits.dtype, device=hits.device)
    pad[: hits.shape[0]] = hits
    out = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, out, dst=dst)
    if rank != dst:
        return None
    return [o[: int(s.item())] for o, s in zip(out, sizes)]


def assemble_tiles(parts, width: int, height: int, world: int, tile: int = 64, owner=None) -> np.ndarray:
    """Scatters gathered per-rank hit records back into screen order (W*H, 4)."""
    full = np.zeros((width * height, 4), np.uint32)
    for r, part in enumerate(parts):
        pix = tile_pixels(width, height, world, r, tile, owner=owner)
        arr = part.cpu().numpy() if hasattr(part, "cpu") else np.asarray(part)
        full[pix] = arr.view(np.uint32).reshape(-1, 4)
    return full


def part_pixels(width: int, height: int, world: int, rank: int, parts: int, tile: int = 64, owner=None):
    """A rank's tiles split into ``parts`` tile-interleaved parts (traced on concurrent streams):
    part s of rank r is virtual rank s * world + r of world * parts, so the union over s is exactly
    tile_pixels(width, height, world, rank) (with a deal ``owner``: virtual_owner)."""
    vo = None if owner is None else virtual_owner(owner, world, parts)
    return [tile_pixels(width, height, world * parts, s * world + rank, tile, owner=vo) for s in range(parts)]


def assemble_parts(gathered, part_sizes, width: int, height: int, world: int, parts: int, tile: int = 64,
                   owner=None) -> np.ndarray:
    """Screen-order hit records from one gathered block per rank: rank r's block holds its parts'
    records back to back (part_sizes[r][s] records each)."""
    virt = [None] * (world * parts)
    for r in range(world):
        arr = gathered[r].cpu().numpy() if hasattr(gathered[r], "cpu") else np.asarray(gathered[r])
        arr = arr.view(np.uint32).reshape(-1, 4)
        o = 0
        for s in range(parts):
            n = int(part_sizes[r][s])
            virt[s * world + r] = arr[o:o + n]
            o += n
    vo = None if owner is None else virtual_owner(owner, world, parts)
    return assemble_tiles(virt, width, height, world * parts, tile, owner=vo)


def n_tiles(width: int, height: int, tile: int = 64) -> int:
    return ((width + tile - 1) // tile) * ((height + tile - 1) // tile)


def spp_part_pixels(width: int, height: int, world: int, rank: int, parts: int, tile: int = 64):
    """``rank``'s share of an ``world``-sample frame, as ``parts`` lists of (sample k, pixel indices).

    Unit u = k * T + t (sample k, tile t of T) goes to rank u % world, so rank r holds, for sample k,
    the tiles t = (r - k * T) mod world (mod world) -- exactly tile_pixels of virtual rank
    (r - k * T) % world -- and every rank holds T units, one frame's worth. Each sample's tiles are
    then split into ``parts`` tile-interleaved parts (part_pixels); part s concatenates them over k."""
    T = n_tiles(width, height, tile)
    out = [[] for _ in range(parts)]
    for k in range(world):
        v = (rank - k * T) % world
        for s, pix in enumerate(part_pixels(width, height, world, v, parts, tile)):
            out[s].append((k, pix))
    return out


def assemble_spp(gathered, width: int, height: int, world: int, parts: int, tile: int = 64) -> np.ndarray:
    """(world, W*H, 4) per-sample screen-order hit records from one gathered block per rank, each
    holding its parts' records back to back in spp_part_pixels order."""
    out = np.zeros((world, width * height, 4), np.uint32)
    for r in range(world):
        arr = gathered[r].cpu().numpy() if hasattr(gathered[r], "cpu") else np.asarray(gathered[r])
        arr = arr.view(np.uint32).reshape(-1, 4)
        o = 0
        for lst in spp_part_pixels(width, height, world, r, parts, tile):
            for k, pix in lst:
                out[k, pix] = arr[o:o + len(pix)]
                o += len(pix)
    return out
