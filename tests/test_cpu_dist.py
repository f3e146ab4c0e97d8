"""Batch-shard logic of upr/dist.py over a world_size-2 gloo group on CPU."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from upr.dist import shard_bounds, gather_shards


def test_shard_bounds_cover_exactly():
    for total in (1, 7, 32, 256, 257):
        for world in (1, 2, 4, 8):
            spans = [shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    full = torch.arange(total * 6, dtype=torch.float32).reshape(total, 2, 3)
    a, b = shard_bounds(total, world, rank)
    got = gather_shards(full[a:b] * 1.0, total)
    q.put((rank, bool(torch.equal(got, full))))
    dist.destroy_process_group()


def test_gloo_gather_world2():
    ctx = mp.get_context("spawn")
    for total in (8, 5):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
        for p in procs:
            p.start()
        res = [q.get(timeout=120) for _ in procs]
        for p in procs:
            p.join(timeout=60)
        assert sorted(res) == [(0, True), (1, True)]


def _grad_worker(rank, world, port, q):
    from types import SimpleNamespace
    from upr.dist import allreduce_grads
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.arange(10, dtype=torch.float32) * (rank + 1)
    opt = SimpleNamespace(flat=SimpleNamespace(grad=g))
    allreduce_grads(opt)
    # mean over ranks of k * (r + 1) = k * (world + 1) / 2
    want = torch.arange(10, dtype=torch.float32) * (world + 1) / 2
    q.put((rank, bool(torch.allclose(opt.flat.grad, want))))
    dist.destroy_process_group()


def test_gloo_allreduce_grads_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_grad_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res) == [(0, True), (1, True)]


def test_bench_gpus2_launches_two_gloo_ranks():
    """`bench.py --gpus 2` run directly is a launcher: it starts torch.distributed.run
    with 2 ranks (here with --dry-run: gloo, CPU step) and rank 0 reports
    n_gpus 2 with the max-over-ranks time; both ranks are distinct processes."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--dry-run", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 3
    ranks = out["ranks"]
    assert sorted(rk for rk, _ in ranks) == [0, 1]
    assert len({pid for _, pid in ranks}) == 2 and os.getpid() not in {pid for _, pid in ranks}
