"""The data-parallel gradient path (GradBucketer) with world_size 2 on gloo/CPU: the
bucketed, hook-launched all-reduce must give every rank the gradient of the global batch."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(16, 300), torch.nn.Tanh(), torch.nn.Linear(300, 200),
                               torch.nn.Tanh(), torch.nn.Linear(200, 4))


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from visual_onoma_to_wave_amd.train import GradBucketer
    m = _model()
    # tiny buckets so several collectives are in flight during backward
    bk = GradBucketer(m.parameters(), bucket_mb=0.05)
    bk.broadcast_parameters(m)
    torch.manual_seed(123)
    x, y = torch.randn(8, 16), torch.randn(8, 4)
    xs, ys = x[rank * 4:(rank + 1) * 4], y[rank * 4:(rank + 1) * 4]
    for _ in range(2):  # two steps: the bucket state resets between steps
        m.zero_grad()
        ((m(xs) - ys) ** 2).mean().backward()
        bk.finish()
    out[rank] = [p.grad.clone() for p in m.parameters()]
    assert len(bk.buckets) >= 3
    dist.destroy_process_group()


def test_bucketed_allreduce_matches_global_batch():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    m = _model()
    torch.manual_seed(123)
    x, y = torch.randn(8, 16), torch.randn(8, 4)
    ((m(x) - y) ** 2).mean().backward()
    for r in range(world):
        for g, p in zip(out[r], m.parameters()):
            torch.testing.assert_close(g, p.grad, rtol=1e-5, atol=1e-6)


def test_unused_parameters_are_identified():
    from helpers import configs
    from visual_onoma_to_wave_amd.model import vTTS
    from visual_onoma_to_wave_amd.train import unused_on_path
    m = vTTS(*configs())
    skip = unused_on_path(m)
    names = {n for n, p in m.named_parameters() if id(p) in skip}
    assert names == {"encoder.src_word_emb.weight", "variance_adaptor.kurt_embedding.weight"}
