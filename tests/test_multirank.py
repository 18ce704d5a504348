"""The N>1 bench path on CPU (gloo, world_size 2): one independent sequence per
rank, MAX-over-ranks timing and the result gather to rank 0."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from dpvo.synthetic import steady_state_edges
        # per-rank work differs (seed = rank); the timing reduction is a MAX
        elapsed = bench.max_over_ranks(1.0 + rank, "cpu")
        pts = torch.full((5, 3), float(rank))
        poses = torch.arange(7.0).repeat(4, 1) + 100 * rank
        got = bench.gather_to_rank0([pts, poses], rank, world)
        ii, jj, kk = steady_state_edges(40, 4, 13, 22, "cpu")
        if rank == 0:
            q.put((elapsed, [[t.tolist() for t in g] for g in got], int(ii.numel())))
        else:
            q.put(None)
    finally:
        dist.destroy_process_group()


def test_two_rank_gather_and_max_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [r for r in res if r is not None]
    assert len(res) == 1
    elapsed, (pts, poses), E = res[0]
    assert elapsed == 2.0
    assert [p[0][0] for p in pts] == [0.0, 1.0]
    assert [p[0][0] for p in poses] == [0.0, 100.0]
    assert E == 497 * 4


@pytest.mark.gpu
def test_bench_main_two_ranks_under_torchrun(tmp_path):
    """bench.main() itself under torch.distributed.run, world_size 2: each
    rank builds its own steady-state tracker (seed = rank), runs the
    graph-replayed update() loop, MAX-over-ranks timing and the result gather
    to rank 0.  Both ranks share the test box's one GPU, so the collectives
    run over gloo (DPVO_BENCH_BACKEND); the driver's 8-GPU run uses RCCL."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DPVO_BENCH_BACKEND="gloo", OMP_NUM_THREADS="4")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(repo, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "1", "--buffer", "72", "--no-cpu-baseline",
           "--e2e-frames", "0"]
    r = subprocess.run(cmd, env=env, cwd=repo, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 prints the one line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak" and line["value"] > 0
    assert line["gather_ms"] >= 0
    assert line["value"] == pytest.approx(2 * 3 / (line["ms_per_step"] * 3 / 1e3), rel=1e-3)
