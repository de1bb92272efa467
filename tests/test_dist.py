"""Multi-process (world_size 2, gloo, CPU) coverage of the multi-GPU path's logic: tile sharding
covers every pixel exactly once, and per-rank traces gathered to rank 0 reassemble into exactly
the single-process frame. The per-rank tracer here is the CPU oracle (test infrastructure); on
the GPU box the same code runs with the HIP engine and the nccl (RCCL) backend."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

import ttdist

HERE = os.path.dirname(os.path.abspath(__file__))


def test_tile_sharding_partitions_the_screen():
    for W, H, world in ((1920, 1080, 8), (1920, 1080, 3), (100, 37, 2), (64, 64, 4)):
        parts = [ttdist.tile_pixels(W, H, world, r) for r in range(world)]
        allp = np.concatenate(parts)
        assert len(allp) == W * H and len(np.unique(allp)) == W * H
        sizes = [len(p) for p in parts]
        assert max(sizes) - min(sizes) <= 64 * 64


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist

    import oracle_ctypes as O
    import tthip
    import ttdist as td

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H = 96, 70
    sc = tthip.single_object_scene(tthip.Mesh.soup(77, 3000, 1.0, 0.08))
    c2w, ip = tthip.unity_camera((0.2, 0.1, 3.0), (0, 0, -1), (0, 1, 0), 55, W, H, 0.3, 1000.0)
    full = O.generate(c2w, ip, W, H, 0.3, 1000.0)
    pix = td.tile_pixels(W, H, world, rank, tile=16)
    mine = np.zeros(2 * len(pix), full.dtype)
    mine[: len(pix)] = full[pix]
    st, _ = O.trace(sc, mine, len(pix), 0, 1000.0, len(pix), 1)
    assert st == 0
    hits = torch.from_numpy(mine["hits"][: len(pix)].astype(np.int64).astype(np.int32))
    parts = td.gather_hits(hits, world, rank)
    if rank == 0:
        got = td.assemble_tiles(parts, W, H, world, tile=16)
        ref = full.copy()
        st, _ = O.trace(sc, ref, W * H, 0, 1000.0, W, H)
        q.put(bool(np.array_equal(got, ref["hits"][: W * H])))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_rank_tile_shard_and_gather():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def test_part_split_partitions_each_rank_and_reassembles():
    """bench.py --parts: a rank's tiles split into tile-interleaved parts traced on concurrent
    streams; the parts cover the rank's pixels exactly and the per-rank blocks (parts back to back)
    reassemble into the screen."""
    W, H = 1920, 1080
    for world, parts in ((2, 2), (8, 2), (4, 3), (8, 3), (1, 2)):
        frame = np.zeros((W * H, 4), np.uint32)
        frame[:, 0] = np.arange(W * H, dtype=np.uint32)  # every pixel's record names its pixel
        blocks, sizes = [], []
        for r in range(world):
            ps = ttdist.part_pixels(W, H, world, r, parts)
            assert np.array_equal(np.sort(np.concatenate(ps)), np.sort(ttdist.tile_pixels(W, H, world, r)))
            blocks.append(np.concatenate([frame[p] for p in ps]))
            sizes.append([len(p) for p in ps])
        got = ttdist.assemble_parts(blocks, sizes, W, H, world, parts)
        assert np.array_equal(got, frame)


def test_spp_units_partition_every_sample_and_balance_ranks():
    """bench.py default at N > 1 (weak scaling): an N-sample frame's (sample, tile) units dealt round-robin
    cover every (sample, pixel) exactly once and give every rank one frame's worth of tiles."""
    W, H = 1920, 1080
    T = ttdist.n_tiles(W, H)
    for world, parts in ((1, 2), (2, 2), (3, 2), (4, 3), (8, 2), (8, 3)):
        seen = np.zeros((world, W * H), np.int32)
        for r in range(world):
            units = ttdist.spp_part_pixels(W, H, world, r, parts)
            assert len(units) == parts
            n_pix = 0
            for lst in units:
                for k, pix in lst:
                    seen[k, pix] += 1
                    n_pix += len(pix)
            # T units per rank: the frame's pixel count up to the partial edge tiles
            assert abs(n_pix - W * H) <= 64 * 64 * world, (world, r, n_pix)
        assert (seen == 1).all()
    # N = 1 is exactly the single-GPU parts layout
    a = [pix for lst in ttdist.spp_part_pixels(W, H, 1, 0, 2) for _, pix in lst]
    b = ttdist.part_pixels(W, H, 1, 0, 2)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert T == 30 * 17


def test_spp_assemble_reorders_gathered_blocks():
    W, H = 200, 130
    for world, parts in ((2, 2), (3, 1), (4, 3), (8, 2)):
        frames = np.zeros((world, W * H, 4), np.uint32)
        frames[:, :, 0] = np.arange(W * H, dtype=np.uint32)[None, :]
        frames[:, :, 1] = np.arange(world, dtype=np.uint32)[:, None]
        blocks = []
        for r in range(world):
            blocks.append(np.concatenate([frames[k, pix] for lst in ttdist.spp_part_pixels(W, H, world, r, parts)
                                          for k, pix in lst]))
        assert np.array_equal(ttdist.assemble_spp(blocks, W, H, world, parts), frames)


def _spp_worker(rank, world, port, q):
    sys.path.insert(0, HERE)
    import torch
    import torch.distributed as dist

    import oracle_ctypes as O
    import tthip
    import ttdist as td

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H, P = 96, 70, 2
    sc = tthip.single_object_scene(tthip.Mesh.soup(78, 3000, 1.0, 0.08))
    c2w, ip = tthip.unity_camera((0.2, 0.1, 3.0), (0, 0, -1), (0, 1, 0), 55, W, H, 0.3, 1000.0)
    samples = [O.generate(c2w, ip, W, H, 0.3, 1000.0, jitter=1, frames=k) for k in range(world)]
    block = []
    for lst in td.spp_part_pixels(W, H, world, rank, P, tile=16):
        for k, pix in lst:
            mine = np.zeros(2 * max(len(pix), 1), samples[0].dtype)
            mine[: len(pix)] = samples[k][pix]
            st, _ = O.trace(sc, mine, len(pix), 0, 1000.0, len(pix), 1)
            assert st == 0
            block.append(mine["hits"][: len(pix)])
    hits = torch.from_numpy(np.concatenate(block).astype(np.int64).astype(np.int32))
    got = td.gather_hits(hits, world, rank)
    if rank == 0:
        frames = td.assemble_spp(got, W, H, world, P, tile=16)
        ok = True
        for k in range(world):
            ref = samples[k].copy()
            st, _ = O.trace(sc, ref, W * H, 0, 1000.0, W, H)
            ok = ok and bool(np.array_equal(frames[k], ref["hits"][: W * H]))
        q.put(ok)
    dist.barrier()
    dist.destroy_process_group()


def _run_spp_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_spp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) is True


def test_gloo_two_rank_spp_shard_and_gather():
    _run_spp_ranks(2)


def test_gloo_eight_rank_spp_shard_and_gather():
    """The largest --gpus the driver runs (N = 8), rehearsed on the CPU: 8 gloo ranks, each traces its
    (sample, tile) units of an 8-sample frame with the oracle, one gather to rank 0, every sample
    reassembled identical to a whole-frame trace."""
    _run_spp_ranks(8)


def test_lpt_deal_covers_every_tile_and_balances():
    """The strong-scaling LPT deal (bench.py --deal lpt): every tile to exactly one rank, the load spread
    within the largest tile's cost, deterministic; per-rank pixel lists and parts partition the screen and
    reassemble to screen order."""
    import ttdist as td

    W, H, world, P = 1920, 1080, 8, 2
    T = td.n_tiles(W, H)
    rng = np.random.default_rng(3)
    chunks = rng.integers(0, 400, (H // 8) * (W // 8)) * (rng.random((H // 8) * (W // 8)) < 0.3)
    costs = td.tile_costs_from_chunks(chunks, W, H)
    assert costs.shape == (T,) and costs.min() >= 24 * 0  # every tile has its cheap-chunk floor
    owner = td.lpt_owner(costs, world)
    assert np.array_equal(owner, td.lpt_owner(costs, world))
    loads = np.bincount(owner, weights=costs, minlength=world)
    assert loads.max() - loads.min() <= costs.max()
    seen = np.zeros(W * H, np.int64)
    frames = np.arange(W * H, dtype=np.uint32)[:, None].repeat(4, 1)
    blocks, sizes = [], []
    for r in range(world):
        parts = td.part_pixels(W, H, world, r, P, owner=owner)
        for pix in parts:
            seen[pix] += 1
        blocks.append(np.concatenate([frames[p] for p in parts]))
        sizes.append([len(p) for p in parts])
    assert np.all(seen == 1)
    assert np.array_equal(td.assemble_parts(blocks, sizes, W, H, world, P, owner=owner), frames)


def test_split_batched_gather_takes_device_blocks_and_reassembles():
    """bench.split_batched_gather: the RCCL gather hands rank 0 DEVICE tensors (one block per rank: its parts back to
    back, each part's B frames back to back); the split must copy them to the host itself (np.concatenate on a
    device tensor raises) and give per frame the blocks assemble_parts takes. Checked with tensors standing in for
    the device blocks (anything with .cpu()) against the frames' own records."""
    import importlib.util

    import torch

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(repo, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    W, H, world, P, B = 192, 128, 2, 2, 3

    class Dev:  # a block that only converts through .cpu(), as a device tensor does
        def __init__(self, t):
            self.t = t

        def cpu(self):
            return self.t

        def __getitem__(self, k):
            return Dev(self.t[k])

    frames = [np.arange(W * H * 4, dtype=np.uint32).reshape(-1, 4) + np.uint32(b * 10_000_000) for b in range(B)]
    blocks, sizes = [], []
    for r in range(world):
        parts = ttdist.part_pixels(W, H, world, r, P)
        rows = [frames[b][pix] for pix in parts for b in range(B)]
        blocks.append(Dev(torch.from_numpy(np.concatenate(rows).view(np.int32))))
        sizes.append([B * len(pix) for pix in parts])
    out = bench.split_batched_gather(blocks, sizes, B)
    assert len(out) == B
    for b, (fb, sb) in enumerate(out):
        assert all(isinstance(x, np.ndarray) for x in fb)
        got = ttdist.assemble_parts(fb, sb, W, H, world, P)
        assert np.array_equal(got, frames[b])
