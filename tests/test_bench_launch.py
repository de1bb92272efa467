"""bench.py's rank launcher: `bench.py --gpus N` without a launcher starts N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torchrun sets them) and exits with
the worst rank's code; under a launcher whose WORLD_SIZE differs from --gpus it refuses.

CPU tests: the launch wiring through TT_BENCH_LAUNCH_CHECK=1 (each rank joins a gloo world, reports
what it sees and exits before any GPU work). GPU test: the whole bench through the self-launch path
with 2 ranks sharing the one GPU over gloo (the driver's 8-GPU node uses RCCL), asserting the
reported world and that the gathered frame equals one GPU's."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE",
                        "TT_BENCH_LAUNCH_CHECK_FAIL_RANK", "TT_BENCH_SELF_LAUNCHED")}
    env.update(kw)
    return env


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def test_self_launch_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3"], env=_env(TT_BENCH_LAUNCH_CHECK="1"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = sorted(_json_lines(r.stdout), key=lambda d: d["rank"])
    assert [d["rank"] for d in recs] == [0, 1, 2]
    for d in recs:
        assert d["world"] == 3 and d["dist_world_size"] == 3 and d["dist_rank"] == d["rank"]
        assert d["local_rank"] == d["rank"] and d["self_launched"]


def test_self_launch_returns_worst_rank_code():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"],
                       env=_env(TT_BENCH_LAUNCH_CHECK="1", TT_BENCH_LAUNCH_CHECK_FAIL_RANK="1"),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])


def test_world_size_mismatch_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"],
                       env=_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT="29555", TT_BENCH_LAUNCH_CHECK="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in (r.stderr + r.stdout)


def test_external_launcher_world_accepted():
    """--gpus equal to the launcher's WORLD_SIZE (or omitted) runs as that rank, no self-launch."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1"],
                       env=_env(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
                                MASTER_PORT=str(_port()), TT_BENCH_LAUNCH_CHECK="1"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    (d,) = _json_lines(r.stdout)
    assert d["world"] == 1 and not d["self_launched"]


def _port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_bench_self_launch_two_ranks_gloo_on_one_gpu():
    """The full bench through the self-launch path: 2 ranks on the one GPU (gloo collectives), the
    headline's strong-scaling tile layout (one 1080p frame's tiles over the ranks, one gather per step); rank 0's JSON line reports 2 GPUs and a gathered frame identical to one GPU
    tracing the whole frame, and the weak-scaling spp layout beside it (a 2-sample frame, same gather)
    identical too."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
                        "--no-shadow", "--no-c5-tiles", "--steady-steps", "0"],
                       env=_env(TT_BENCH_DIST_BACKEND="gloo"), capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    (d,) = _json_lines(r.stdout)
    assert d["n_gpus"] == 2
    c = d["config"]
    assert c["dist_world_size"] == 2 and c["launcher"] == "bench.py self-launch"
    assert c["gather_identical_to_1gpu"] is True
    assert d["scaling"] == "strong" and c["samples_per_frame"] == 1
    fps = c["frames_per_step"]  # frames each launch traces (bench.py --batch; 4 at N > 1)
    assert fps >= 1 and 4_000_000 < c["rays_per_step_all_ranks"] / fps < 4_200_000  # 1080p frames, primary + bounce 1
    st = c["aux_strong_tiles"]
    assert st["scaling"] == "strong" and st["gather_identical_to_1gpu"] is True
    assert st["tile_deal"]["deal"] == "round-robin"
    assert 4_000_000 < st["rays_per_frame_all_ranks"] < 4_200_000
    assert st["frame_slots"] >= 1 and 4_000_000 < st["n1_rays_per_frame"] < 4_200_000
    assert st["frames_per_launch"] == fps
    assert 0.0 < st["efficiency"]
    assert abs(st["efficiency"] - st["n1_ms_per_frame"] / (2 * st["ms_per_frame"])) < 0.01
    w = c["aux_spp_weak"]
    assert w["scaling"] == "weak" and w["samples_per_frame"] == 2 and w["gather_identical_to_1gpu"] is True
