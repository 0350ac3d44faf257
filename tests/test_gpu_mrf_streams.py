"""The conv-path MRF stage (C = 256) runs its three ResBlock chains on concurrent streams
(hifigan/models.py ``Generator._mrf_concurrent``); the chains' accumulations into the MRF sum are
ordered by events, so the output must equal the sequential loop's bit for bit -- eagerly, under a
HIP-graph capture, and with the vocoder on a non-default stream (the bench's pipeline)."""

import pytest
import torch

from helpers import hifigan_arrays, hifigan_h
from weights import load_into

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gen(device):
    from visual_onoma_to_wave_amd import hifigan
    g = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    load_into(g, hifigan_arrays())
    g.eval()
    g.remove_weight_norm()
    return g.to(device)


def _mel(B, T, seed):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(B, T, 80, generator=g) * 1.5 - 4.0).cuda()


def _run(gen, mel, concurrent):
    from visual_onoma_to_wave_amd.hifigan import models
    old = models.MRF_STREAMS
    models.MRF_STREAMS = concurrent
    try:
        with torch.no_grad():
            return gen.run(mel)
    finally:
        models.MRF_STREAMS = old


@pytest.mark.parametrize("B,T", [(1, 7), (3, 64), (32, 160)])
def test_concurrent_mrf_matches_sequential(gen, B, T):
    mel = _mel(B, T, B * 1000 + T)
    ref = _run(gen, mel, False)
    for _ in range(2):
        out = _run(gen, mel, True)
        torch.cuda.synchronize()
        assert torch.isfinite(out).all()
        assert torch.equal(out, ref)


def test_concurrent_mrf_on_side_stream_and_graph(gen):
    mel = _mel(4, 48, 7)
    ref = _run(gen, mel, False)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        out = _run(gen, mel, True)
    torch.cuda.current_stream().wait_stream(s)
    assert torch.equal(out, ref)
    # capture the concurrent form and replay it back to back
    static = mel.clone()
    _run(gen, static, True)  # warm the pack cache outside the capture
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        gout = _run(gen, static, True)
    for seed in (11, 12, 13):
        static.copy_(_mel(4, 48, seed))
        graph.replay()
        want = _run(gen, static, False)
        torch.cuda.synchronize()
        assert torch.equal(gout, want)
