"""bench.py's live kernel timing (profiling.KernelTimer): an MRF stage's consecutive ResBlock
launches are bracketed by one event pair (`group`); launch counts, FLOPs and the elapsed time
must still come out per stage."""
import pytest
import torch

from helpers import hifigan_arrays, hifigan_h
from weights import load_into

pytestmark = pytest.mark.gpu


def test_grouped_stage_timing(device):
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.profiling import KernelTimer
    gen = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    load_into(gen, hifigan_arrays())
    gen.eval()
    gen.remove_weight_norm()
    gen = gen.to(device)
    gen.set_compute_dtype(torch.bfloat16)
    mel = torch.randn(2, 64, 80, device=device)
    tags = [f"mrf_s{i}" for i in range(4)]
    with torch.no_grad():
        ref = gen.run(mel)
        timer = KernelTimer(tags)
        with timer:
            for _ in range(2):
                wav = gen.run(mel)
    assert torch.equal(wav, ref)
    ks = timer.summary()
    assert set(ks) == set(tags)
    assert not timer.pending  # no per-launch event pairs inside the groups
    assert ks["mrf_s0"]["launches"] == 2 * 18   # C = 256: two conv launches per (c1, c2) pair
    for t in tags[1:]:
        assert ks[t]["launches"] == 2 * 7      # 3 + 3 fused pairs (k = 7, 11) + 1 fused k = 3 block
    for d in ks.values():
        assert d["avg_ms"] > 0 and d["flops_per_launch"] > 0
