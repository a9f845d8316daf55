"""bench.py's whole-job accounting (the headline `value`) and its rank launcher.

The reference's SPS numerator is `global_step`, the mask-true agent steps
(puffer_phc/clean_pufferl/core.py:135-138, structs.py:354).  Under data parallelism evaluate()
already sums it over ranks, so the ppo mode must take it once; the env / rollout modes count
per-rank steps, which are summed.  The GPU test runs `bench.py --gpus 2` with the gloo backend
(two ranks on the one leased GPU, launched by bench.py itself) and checks the JSON line's value
against the rows the two ranks collected.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench

    return bench


def test_whole_job_steps_ppo_counts_once():
    b = _bench()
    # every rank reports the rank-summed global_step delta: taken once, not world x
    assert b.whole_job_steps([262144.0, 262144.0], True, 2) == 262144.0
    assert b.whole_job_steps([131072.0], True, 1) == 131072.0
    with pytest.raises(ValueError):
        b.whole_job_steps([262144.0, 262000.0], True, 2)  # ranks must agree


def test_whole_job_steps_env_modes_sum():
    b = _bench()
    assert b.whole_job_steps([4096.0 * 200] * 8, False, 8) == 8 * 4096.0 * 200
    with pytest.raises(ValueError):
        b.whole_job_steps([1.0], False, 2)


def test_launcher_command_is_torchrun_child(monkeypatch):
    """launch_ranks starts torch.distributed.run as a child on the loopback rendezvous and
    forwards this script's arguments (no exec of the parent)."""
    b = _bench()
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, *a, **k):
        seen["cmd"] = cmd
        return R()

    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    assert b.launch_ranks(4) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "2"] and cmd[-5].endswith("bench.py")


@pytest.mark.gpu
def test_two_rank_gloo_bench_reports_rows_over_wall():
    env = dict(os.environ, PHC_DIST_BACKEND="gloo", HSA_ENABLE_IPC_MODE_LEGACY="0")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--mode", "ppo", "--steps", "1",
           "--warmup", "1", "--envs", "512", "--batch-size", "8192", "--minibatch-size", "2048",
           "--no-cpu-baseline", "--dp-mode", "split"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_envs"] == 1024
    dp = out["config"]["dp"]  # the exposed all-reduce wait per minibatch backward
    assert set(dp) == set(_bench().DP_FIELDS)
    assert dp["mode"] == "split" and dp["minibatches_timed"] >= 4 and dp["backend"] == "gloo"
    assert dp["allreduce_exposed_ms_per_minibatch_max_rank"] >= dp["allreduce_exposed_ms_per_minibatch_rank0"] >= 0
    rows = out["config"]["env_steps_timed"]
    # each rank collects >= its batch of mask-true rows per iteration (plus the last step's
    # overflow), so the whole job is ~2 x 8192, not 4 x
    assert 2 * 8192 <= rows < 2 * 8192 + 2 * 512
    wall_s = out["ms_per_step"] * out["steps"] / 1e3
    assert out["value"] == pytest.approx(rows / wall_s, rel=1e-9)


def _dp_worker(rank, world, port, root, out):
    import torch
    import torch.distributed as dist

    sys.path.insert(0, root)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank r waited 0.5 + r ms per backward over 8 minibatches (rank 1 reports none: a rank with no
        # timed backward contributes 0 to the max)
        exp = 0.5 + rank if rank != 1 else None
        dp = bench.dp_summary("split", exp, 8, 4 * 1000, "cpu")
        mine = torch.tensor([131072.0 + 17], dtype=torch.float64)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        total = bench.whole_job_steps([float(c) for c in every], True, world)
        out.put((rank, dp, total))
    finally:
        dist.destroy_process_group()


def test_dp_summary_world3_gloo_cpu():
    """config.dp over three gloo ranks on the CPU: every field present, the slowest rank's exposed
    wait is the max over ranks, the backend is named, and the ppo count is taken once."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dp_worker, args=(r, 3, port, ROOT, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    fields = _bench().DP_FIELDS
    for rank, dp, total in res:
        assert tuple(dp) == fields
        assert dp["backend"] == "gloo" and dp["mode"] == "split" and dp["minibatches_timed"] == 8
        assert dp["allreduce_exposed_ms_per_minibatch_max_rank"] == 2.5
        assert dp["allreduce_exposed_ms_per_minibatch_rank0"] == (0.5 + rank if rank != 1 else None)
        assert dp["grad_bytes_per_minibatch"] == 4000
        assert total == 131072.0 + 17
