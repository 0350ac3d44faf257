"""Data-parallel C4 training on the GPU (reference: scripts/04_train.py:75,128-141, where
``nn.DataParallel`` splits the batch over GPUs and reduce-adds the gradients).

* two ranks (gloo, CUDA tensors, both on cuda:0 -- the one-GPU box): each runs the real vTTS
  train step on its half of the batch with ``GradBucketer``; every rank's averaged gradients must
  equal the mean of the per-shard gradients of a single process (BatchNorm statistics are per
  shard, as they are per replica under DataParallel);
* one rank on RCCL: the whole step including the bucketed all-reduces captured as one HIP graph
  (``GraphedTrainStep(bucketer=...)``) against the eager bucketed step.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from helpers import configs, golden, vtts_arrays
from weights import load_into

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _model(dev, prec="fp32", tc_over=None):
    from visual_onoma_to_wave_amd.model import vTTS
    pc, mc, tc = configs()
    if tc_over:
        tc = dict(tc)
        tc["optimizer"] = dict(tc["optimizer"], **tc_over)
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(dev).train().set_precision(prec)
    for mod in m.modules():
        if isinstance(mod, torch.nn.Dropout):
            mod.p = 0.0
    m.postnet.dropout_p = 0.0
    for vp in (m.variance_adaptor.duration_predictor, m.variance_adaptor.energy_predictor):
        vp.dropout = 0.0
    return m, (pc, mc, tc)


def _batch(dev, sl=slice(None)):
    g = golden("vtts_tf")
    t = lambda k: torch.from_numpy(np.array(g[k])[sl]).to(dev)  # noqa: E731
    return (None, t("in_audiotypes"), t("in_texts"), t("in_src_lens"), int(g["in_max_src_len"]), t("in_mels"),
            t("in_mel_lens"), int(g["in_max_mel_len"]), t("in_e_targets"), None, t("in_d_targets"),
            t("in_images"), None)


def _shard_grads(dev, shard):
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss
    m, _ = _model(dev)
    batch = _batch(dev, slice(shard, shard + 1))
    out = m(*(batch[1:]), True)
    FastSpeech2Loss()(batch, out)[0].backward()
    return {n: p.grad.detach().cpu().clone() for n, p in m.named_parameters() if p.grad is not None}


def _gloo_worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss
    from visual_onoma_to_wave_amd.train import GradBucketer, unused_on_path
    m, _ = _model(dev)
    skip = unused_on_path(m)
    bk = GradBucketer([p for p in m.parameters() if id(p) not in skip], bucket_mb=8.0)
    bk.broadcast_parameters(m)
    batch = _batch(dev, slice(rank, rank + 1))
    out_ = m(*(batch[1:]), True)
    FastSpeech2Loss()(batch, out_)[0].backward()
    bk.finish()
    torch.cuda.synchronize()
    out[rank] = ({n: p.grad.detach().cpu().clone() for n, p in m.named_parameters() if p.grad is not None},
                 len(bk.buckets))
    dist.destroy_process_group()


def test_bucketed_ddp_vtts_grads_match_shard_mean(device):
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_gloo_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    ref = [_shard_grads(device, r) for r in range(world)]
    for r in range(world):
        grads, n_buckets = out[r]
        assert n_buckets >= 10
        assert set(grads) == set(ref[0]) or set(grads) >= set(ref[0])
        bad = []
        for n, g0 in ref[0].items():
            want = (g0 + ref[1][n]) / 2
            err = float((grads[n] - want).norm())
            if err > 1e-4 * float(want.norm()) + 1e-6:
                bad.append((n, err, float(want.norm())))
        assert not bad, bad[:8]


def _rccl_graph_worker(rank, world, port, out, bound=True):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if bound:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:  # default group not bound to a device: the graph group must still connect eagerly
        dist.init_process_group("nccl", rank=rank, world_size=world)
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim
    from visual_onoma_to_wave_amd.train import GradBucketer, GraphedTrainStep, train_step, unused_on_path
    res = []
    for graphed in (False, True):
        m, (pc, mc, tc) = _model(dev, tc_over=dict(warm_up_step=10, init_lr=1e-3))
        skip = unused_on_path(m)
        bk = GradBucketer([p for p in m.parameters() if id(p) not in skip], bucket_mb=8.0,
                          comm_dtype=None)
        opt = ScheduledOptim(m, tc, mc, 0, capturable=graphed)
        batch = _batch(dev)
        losses = []
        if graphed:
            run = GraphedTrainStep(m, opt, FastSpeech2Loss(), warmup=2, bucketer=bk)
            for _ in range(6):
                losses.append(run(batch)[0].detach().clone())
        else:
            for _ in range(6):
                losses.append(train_step(m, opt, FastSpeech2Loss(), batch, bucketer=bk)[0].detach().clone())
        torch.cuda.synchronize()
        res.append(([float(x) for x in losses], torch.cat([p.detach().flatten().cpu() for p in m.parameters()])))
    out[rank] = res
    dist.destroy_process_group()


@pytest.mark.parametrize("bound", [True, False])
def test_graphed_ddp_step_rccl_matches_eager(device, bound):
    """The bucketed RCCL all-reduce captured inside the HIP graph of the whole step (one rank:
    the collective is a real RCCL launch on the side-stream branch of the graph), with the default
    process group bound to the device (init_process_group(device_id=...)) and without (the graph
    group's communicator is then connected eagerly by new_group(device_id=...), not inside the
    capture)."""
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_rccl_graph_worker, args=(1, _free_port(), out, bound), nprocs=1, join=True)
    (le, pe), (lg, pg) = out[0]
    assert np.isfinite(lg).all()
    p_err = float((pg - pe).norm() / pe.norm())
    print(f"graphed DDP vs eager DDP: params {p_err:.2e}, losses {le} vs {lg}")
    assert p_err < 1e-3
    np.testing.assert_allclose(lg, le, rtol=1e-3)
