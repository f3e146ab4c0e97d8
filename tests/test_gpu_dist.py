"""RCCL (torch.distributed "nccl" backend on ROCm) paths of upr/dist.py on the
MI355X at world_size 1 (run with `-m gpu`): gather_shards through
all_gather_into_tensor and allreduce_grads through all_reduce of the flat
gradient buffer.  The world_size-2 logic is covered on CPU (gloo,
tests/test_cpu_dist.py); 8-GPU runs are the driver's scaling bench."""
import os
import socket

import pytest
import torch
import torch.distributed as dist

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a ROCm device")]


@pytest.fixture(scope="module")
def nccl_group():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def test_gather_shards_rccl(nccl_group):
    from upr.dist import gather_shards, shard_bounds
    full = torch.rand(5, 3, 16, 24, device="cuda").half()
    a, b = shard_bounds(5, 1, 0)
    got = gather_shards(full[a:b], 5)
    torch.cuda.synchronize()
    assert got.is_cuda and got.dtype == torch.float16 and torch.equal(got, full)


def test_sharded_forward_collect_rccl(nccl_group):
    from models.model import UP_Retinex
    from upr.dist import sharded_forward
    torch.manual_seed(0)
    m = UP_Retinex(use_preact=False, use_aspp=False).eval().to("cuda")
    x = torch.rand(2, 3, 32, 32, device="cuda")
    enh, _, _ = sharded_forward(m, x, 2, collect=True, collect_dtype=torch.float16)
    with torch.no_grad():
        ref = m(x)[0]
    assert torch.equal(enh, ref.half())


def test_allreduce_grads_rccl(nccl_group):
    from types import SimpleNamespace
    from upr.dist import allreduce_grads
    g = torch.arange(1000, dtype=torch.float32, device="cuda")
    opt = SimpleNamespace(flat=SimpleNamespace(grad=g.clone()))
    allreduce_grads(opt)
    torch.cuda.synchronize()
    assert torch.equal(opt.flat.grad, g)  # mean over one rank
