"""Batch-shard logic of upr/dist.py over a world_size-2 gloo group on CPU."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from upr.dist import shard_bounds, gather_shards, gather_to_rank0


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
    ok = bool(torch.equal(got, full))
    g0 = gather_to_rank0(full[a:b] * 1.0, total)
    ok = ok and (bool(torch.equal(g0, full)) if rank == 0 else g0 is None)
    q.put((rank, ok))
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


def _bench_json(args):
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + args, capture_output=True, text=True,
                       timeout=240, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_gpus2_line_carries_evidence_keys():
    """An N>1 line carries rank 0's parity, the roofline object and the nested
    fp16 object; cpu_baseline and train_amp are N=1 only; --collect rank0 runs
    the gather-to-rank-0 collect through the same timed loop (gloo here)."""
    out = _bench_json(["--gpus", "2", "--dry-run", "--steps", "2", "--warmup", "1", "--collect", "rank0"])
    assert out["n_gpus"] == 2
    for k in ("roofline", "parity", "fp16_preact_aspp", "config"):
        assert k in out, k
    assert "parity" in out["fp16_preact_aspp"]
    assert "cpu_baseline" not in out and "train_amp" not in out
    assert "collect=rank0" in out["config"]["parallelism"]


def test_bench_n1_line_carries_cpu_and_train_keys():
    out = _bench_json(["--dry-run", "--steps", "2", "--warmup", "1"])
    for k in ("roofline", "parity", "cpu_baseline", "fp16_preact_aspp", "train_amp"):
        assert k in out, k
    ci = out["cpu_baseline"]["cpu"]
    assert ci["threads"] >= 1 and "cpu_model" in ci and ci["os_cpu_count"] >= ci["threads"]
