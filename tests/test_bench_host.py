"""Host-side pieces of bench.py (no GPU): the C3 strong-scaling split that the
default run's c3_strong leg and --total-tiles use must partition the 64 tiles
exactly as the library's TileShardedSMC does (smcdet_amd.distributed), so the
union of the ranks' work at N = 2, 4, 8 is the one-GPU workload."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from smcdet_amd.distributed import shard_tiles  # noqa: E402


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 8, 64])
def test_c3_split_partitions_tiles_like_the_library(world):
    total = bench.C3_TILES
    seen = []
    for rank in range(world):
        ids = bench.shard(total, world, rank)
        a, b = shard_tiles(total, world, rank)
        assert ids == list(range(a, b))
        assert ids, "every rank owns at least one tile"
        seen += ids
    assert seen == list(range(total))


def test_c3_leg_is_part_of_the_default_run():
    old = sys.argv
    try:
        sys.argv = ["bench.py"]
        args = bench.parse()
    finally:
        sys.argv = old
    # the leg runs for the default C2 command (c3_leg's guard in main)
    assert (args.workload, args.kernel, args.total_tiles, args.tiles_per_gpu,
            args.no_c3) == ("c2", "mh", 0, 1, False)


def _torchrun_rehearsal(extra, world=2):
    """bench.py under a 2-rank gloo torchrun with --host-rehearsal (stub
    sampler, no GPU): the driver's N > 1 command, minus the kernels."""
    import json
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, SMCDET_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--host-rehearsal",
           "--particles", "64", "--steps", "4", "--warmup", "1"] + extra
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints the one JSON line
    return json.loads(lines[0])


def test_torchrun_two_ranks_c3_strong_scaling_line():
    """--total-tiles 64 over 2 ranks: 32 tiles each (bench.shard), the timed
    region bracketed by barriers, its MAX over ranks (rank 1 sleeps twice as
    long per tile) in ms_per_step, and value = all 64 tiles' particle-steps
    over that time."""
    d = _torchrun_rehearsal(["--total-tiles", "64", "--no-c3"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["tiles_per_gpu"] == 32
    steps = d["steps"]
    assert steps == 4
    # rank 1: 32 tiles x 2 ms per step; the MAX over ranks is its time
    assert d["ms_per_step"] >= 64.0 * 0.95, d["ms_per_step"]
    np_ = d["config"]["particles"] * d["config"]["mh_iters"]
    assert abs(d["value"] - 64 * np_ / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]
    assert "cpu_baseline" not in d  # world > 1: no CPU baseline


def test_torchrun_two_ranks_default_line_with_c3_leg_and_gather():
    """The default C2 command at N = 2: weak scaling (one tile per rank), the
    rank-0-only vs_reference comparisons, and the C3 leg's catalog gather
    (64 tiles -> [8, 8, ...] on rank 0 through gloo)."""
    d = _torchrun_rehearsal([])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    np_ = d["config"]["particles"] * d["config"]["mh_iters"]
    assert abs(d["value"] - 2 * np_ / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]
    assert d["ms_per_step"] >= 2.0 * 0.95  # rank 1's 2 ms per step
    for k in ("vs_reference", "vs_oracle_k100", "vs_reference_k20", "vs_reference_n512"):
        assert d["smc"][k] == {"rehearsal": d["smc"][k]["rehearsal"]}
        assert d["smc"][k]["rehearsal"].endswith("on rank 0")
    c3 = d["c3_strong"]
    assert c3["scaling"] == "strong" and c3["n_gpus"] == 2
    assert c3["config"]["tiles_per_gpu_rank0"] == 32
    g = c3["catalog_gather"]
    assert g["backend"] == "gloo"
    assert g["gathered_shape_locs"] == [8, 8, d["config"]["particles"], 10, 2]
    assert g["bytes_per_rank"] > 0


def test_torchrun_eight_ranks_default_line():
    """The driver's N = 8 command, rehearsed on the CPU: one tile per rank
    (weak scaling), MAX over ranks (rank 7 sleeps 8 ms per step), the C3 leg at
    8 tiles per rank with its catalog gather to [8, 8, ...] on rank 0, and the
    rank-0-only fields."""
    d = _torchrun_rehearsal(["--steps", "3"], world=8)
    assert d["n_gpus"] == 8 and d["scaling"] == "weak"
    assert d["ms_per_step"] >= 8.0 * 0.95, d["ms_per_step"]
    np_ = d["config"]["particles"] * d["config"]["mh_iters"]
    assert abs(d["value"] - 8 * np_ / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]
    c3 = d["c3_strong"]
    assert c3["n_gpus"] == 8 and c3["config"]["tiles_per_gpu_rank0"] == 8
    # rank 7: 8 tiles x 8 ms per step
    assert c3["ms_per_step"] >= 64.0 * 0.95, c3["ms_per_step"]
    assert c3["catalog_gather"]["gathered_shape_locs"] == [8, 8, d["config"]["particles"], 10, 2]
    assert "cpu_baseline" not in d
    assert d["smc"]["vs_reference"]["rehearsal"].endswith("on rank 0")


def test_torchrun_seven_ranks_uneven_c3_shares():
    """64 tiles over 7 ranks: rank 0 owns 10 tiles, ranks 1..6 own 9
    (bench.shard = distributed.shard_tiles); the MAX over ranks is rank 6's
    9 tiles x 7 ms per step, and value counts all 64 tiles."""
    d = _torchrun_rehearsal(["--total-tiles", "64", "--no-c3", "--steps", "3"], world=7)
    assert d["n_gpus"] == 7 and d["scaling"] == "strong"
    assert d["config"]["tiles_per_gpu"] == 10
    assert [len(bench.shard(64, 7, r)) for r in range(7)] == [10] + [9] * 6
    assert d["ms_per_step"] >= 63.0 * 0.95, d["ms_per_step"]
    np_ = d["config"]["particles"] * d["config"]["mh_iters"]
    assert abs(d["value"] - 64 * np_ / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]


def test_gpus_flag_launches_ranks_as_a_child():
    """`python bench.py --gpus 2` without torchrun starts the driver's torchrun
    command as a child process (bench.launch_ranks) and prints its one line."""
    import json
    import subprocess
    env = dict(os.environ, SMCDET_DIST_BACKEND="gloo", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--host-rehearsal", "--particles", "64", "--steps", "3", "--warmup", "1",
                        "--no-c3"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert json.loads(lines[0])["n_gpus"] == 2


def test_gpus_flag_mismatch_fails_loudly():
    """A launcher's WORLD_SIZE that disagrees with --gpus is an error (exit
    status != 0, message on stderr), never a silent one-rank line."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="3", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--host-rehearsal"], env=env, cwd=ROOT, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0
    assert "--gpus 2" in r.stderr and "WORLD_SIZE=3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
