"""ttlayout.FrameLayout's frame -> (slot, cycle position, sample) arithmetic, on the CPU (no engine: the
object is built without __init__). bench.py at N > 1 cycles every frame slot through --cycle samples, so
a costly ray recurs in one frame of `cycle` on its slot; these checks pin which sample each frame traces."""
import ttlayout


class _Part:
    def __init__(self, n, nb_r):
        self.n, self.nb_r = n, nb_r


def _layout(F, R, stride, parts=None):
    lay = ttlayout.FrameLayout.__new__(ttlayout.FrameLayout)
    lay.F, lay.R, lay.stride, lay.k = F, R, stride, 0
    lay.slots = parts if parts is not None else [[_Part(10, [0] * R)] for _ in range(F)]
    return lay


def test_cycle_one_is_the_fixed_slot_sample():
    lay = _layout(F=3, R=1, stride=1)
    assert [lay.frame_sample(k, 0) for k in range(7)] == [0, 1, 2, 0, 1, 2, 0]
    assert [lay.cycle_of(k) for k in range(7)] == [0] * 7
    lay0 = _layout(F=3, R=1, stride=0)  # replicated: one sample everywhere
    assert {lay0.frame_sample(k, 4) for k in range(9)} == {4}


def test_cycle_spreads_samples_over_a_slots_frames():
    F, R = 6, 6
    lay = _layout(F=F, R=R, stride=1)
    samples = [lay.frame_sample(k, 0) for k in range(F * R)]
    assert sorted(samples) == list(range(F * R))  # every (slot, cycle) pair its own sample
    for f in range(F):  # a slot's successive frames trace R different samples, then repeat
        mine = [lay.frame_sample(k, 0) for k in range(f, 3 * F * R, F)]
        assert len(set(mine[:R])) == R and mine[R:2 * R] == mine[:R]
    # a sample recurs once every F * R frames, always on the same slot
    k0 = samples.index(17)
    assert all(lay.frame_sample(k, 0) != 17 for k in range(k0 + 1, k0 + F * R))
    assert lay.frame_sample(k0 + F * R, 0) == 17


def test_rays_in_frames_follow_the_cycle():
    F, R = 2, 3
    parts = [[_Part(100, [10 * (f + 1) + r for r in range(R)])] for f in range(F)]
    lay = _layout(F=F, R=R, stride=1, parts=parts)
    want = sum(100 + 10 * ((k % F) + 1) + (k // F) % R for k in range(4, 17))
    assert lay.rays_in_frames(4, 17) == want
    lay.k = 9
    assert lay.last_slot() == 0 and lay.last_sample(0) == lay.frame_sample(8, 0) == 0 + F * 1


def test_batched_frames_each_trace_their_own_sample():
    # bench.py --batch B at N > 1: a plan names samples 0..B-1 per part and slot_stride = B, so frame j of a
    # launch on slot f in cycle position r traces j + B (f + F r): B F R distinct samples, none shared
    F, R, B = 3, 2, 2
    lay = _layout(F=F, R=R, stride=B)
    seen = [lay.sample_of(f, j, r) for r in range(R) for f in range(F) for j in range(B)]
    assert sorted(seen) == list(range(F * R * B))
    assert lay.sample_of(2, 1, 1) == 1 + B * (2 + F * 1)


def test_split_batched_gather_recovers_every_frame():
    import numpy as np

    import bench

    B, sizes_frame = 2, [[5, 3], [4]]  # two ranks: rank 0 two parts, rank 1 one part (per-frame record counts)
    frames = [[[np.full((n, 4), 100 * b + 10 * r + p, np.uint32) for p, n in enumerate(ns)]
               for r, ns in enumerate(sizes_frame)] for b in range(B)]
    blocks, sizes = [], []
    for r, ns in enumerate(sizes_frame):  # each part's records: the B frames back to back
        blocks.append(np.concatenate([np.concatenate([frames[b][r][p] for b in range(B)]) for p in range(len(ns))]))
        sizes.append([B * n for n in ns])
    out = bench.split_batched_gather(blocks, sizes, B)
    assert len(out) == B
    for b, (fb, sb) in enumerate(out):
        assert sb == sizes_frame
        for r in range(len(sizes_frame)):
            assert np.array_equal(fb[r], np.concatenate(frames[b][r]))
