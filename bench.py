#!/usr/bin/env python3
"""End-to-end visual-onomatopoeia -> 22.05 kHz waveform throughput on MI355X.

One step = one batch of B synthetic rendered-glyph strips (B x 1 x 24 x 102*T_src, T_src=12)
through the acoustic model (teacher-forced durations summing to T_mel=512 frames, predicted
energy) and the HiFi-GAN V1 generator on its postnet mel
(config C3 shape per utterance) -> B x 131,072 samples.  Inputs are resident in HBM
before the timed region.  Multi-GPU: one process per GPU (torchrun), every rank
synthesises its own batch (utterances are independent: replicas, no data-path
collective), only the timing uses a barrier and a MAX all-reduce.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--precision mixed]

Prints ONE JSON line (rank 0) with the metric of BASELINE.json, the dominant kernel's
roofline (HIP events on the launching stream over the timed region) and the CPU
baseline (the oracle restatement timed on this host, bounded sample).
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

SR = 22050
HOP = 256
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (no sparsity)
F32_PEAK_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--src-len", type=int, default=12)
    ap.add_argument("--mel-len", type=int, default=512)
    ap.add_argument("--precision", default="mixed", choices=["mixed", "bf16", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="train / gan modes: eager steps instead of one HIP graph")
    ap.add_argument("--mode", default="infer", choices=["infer", "train", "gan"],
                    help="infer: end-to-end synthesis (headline); train: C4 training step (DDP); "
                         "gan: C5 HiFi-GAN training step (DDP)")
    return ap.parse_args()


def bench_train(a, dev, rank, world, dist):
    """C4: scripts/04_train.py step (teacher-forced forward, FastSpeech2Loss, backward with the
    bucketed RCCL all-reduce, clip 1.0, Adam + schedule) on B utterances per GPU."""
    from helpers import configs, vtts_arrays
    from weights import load_into
    from visual_onoma_to_wave_amd import synth
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import GradBucketer, train_step, unused_on_path
    pc, mc, tc = configs()
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(dev).train().set_precision(a.precision)
    graphed = dist is None and not a.no_graph  # one process: the whole step as a HIP graph replay
    opt = ScheduledOptim(m, tc, mc, 0, capturable=graphed)
    bk = None
    if dist:
        skip = unused_on_path(m)
        bk = GradBucketer([p for p in m.parameters() if id(p) not in skip])
        bk.broadcast_parameters(m)
    b = synth.acoustic_batch(1234 + rank, a.batch, a.src_len, a.mel_len)
    t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
             t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
    loss_fn = FastSpeech2Loss()
    if graphed:
        from visual_onoma_to_wave_amd.train import GraphedTrainStep
        run = GraphedTrainStep(m, opt, loss_fn)
    else:
        def run(bt):
            return train_step(m, opt, loss_fn, bt, bucketer=bk)
    for _ in range(a.warmup):
        run(batch)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        losses = run(batch)
        if os.environ.get("VO_BENCH_DEBUG"):
            print("loss", [round(float(v.detach()), 4) for v in losses[:6]], file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    frames = a.batch * a.mel_len * a.steps * world
    if rank == 0:
        print(json.dumps({
            "metric": "C4 training mel-frames/sec (FastSpeech2 + variance loss, DDP)", "value": round(frames / elapsed, 1),
            "unit": "mel-frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": a.precision, "data": "synthetic",
            "final_loss": round(float(losses[0]), 5), "hip_graph": graphed,
            "config": {"workload": "C4 train step", "per_gpu_batch": a.batch, "global_batch": a.batch * world,
                       "seq_len": a.mel_len, "src_len": a.src_len, "parallelism": f"dp{world} (RCCL bucketed all-reduce)"}}))


def bench_gan(a, dev, rank, world, dist):
    """C5: HiFi-GAN V1 training step (generator + MPD + MSD, D step then G step with adversarial,
    feature-matching and 45 x mel-L1 losses, AdamW) on B segments of 8192 samples per GPU
    (scripts/hifigan/config.json: batch 16, segment 8192)."""
    from helpers import hifigan_arrays, hifigan_h
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.hifigan.discriminators import MelLoss
    h = hifigan.AttrDict(hifigan_h())
    g = hifigan.Generator(h)
    load_into(g, hifigan_arrays())
    g = g.to(dev)
    torch.manual_seed(1234)  # identical discriminator init on every rank (broadcast anyway)
    graphed = dist is None and not a.no_graph  # one process: the whole step as a HIP graph replay
    tr = hifigan.HifiGanTrainer(g, h, distributed=dist is not None, device=dev, graphed=graphed)
    run = tr.step_graphed if graphed else tr.step
    tr.set_compute_dtype(torch.float32 if a.precision == "fp32" else torch.bfloat16)
    B, seg = a.batch, h.segment_size
    gen = torch.Generator().manual_seed(99 + rank)
    t = torch.arange(seg, dtype=torch.float32) / h.sampling_rate
    f0 = 110.0 + 330.0 * torch.rand(B, 1, generator=gen)
    y = (0.3 * torch.sin(2 * np.pi * f0 * t) + 0.05 * torch.randn(B, seg, generator=gen)).to(dev)
    with torch.no_grad():
        x = MelLoss(h.n_fft, h.num_mels, h.sampling_rate, h.hop_size, h.win_size, h.fmin, h.fmax).to(dev).mel(y)
    x = x.transpose(1, 2).contiguous()  # (B, 32, 80) channels-last generator input
    for _ in range(a.warmup):
        run(x, y)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        losses = run(x, y)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    samples = B * seg * a.steps * world
    if rank == 0:
        print(json.dumps({
            "metric": "C5 HiFi-GAN training audio samples/sec (G + MPD + MSD, DDP)", "value": round(samples / elapsed, 1),
            "unit": "audio samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16" if a.precision != "fp32" else "f32",
            "data": "synthetic (sinusoid + noise segments, their mel as generator input)",
            "losses": {k: round(float(v), 4) for k, v in losses.items()},
            "hip_graph": graphed,
            "config": {"workload": "C5 HiFi-GAN V1 train step", "per_gpu_batch": B, "global_batch": B * world,
                       "segment": seg, "parallelism": f"dp{world} (RCCL bucketed all-reduce, G and D)"}}))


def build_models(device, precision):
    from helpers import configs, hifigan_arrays, hifigan_h, vtts_arrays
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.model import vTTS
    m = vTTS(*configs())
    load_into(m, vtts_arrays())
    m = m.to(device).eval().set_precision(precision)
    g = hifigan.Generator(hifigan.AttrDict(hifigan_h()))
    load_into(g, hifigan_arrays())
    g.eval()
    g.remove_weight_norm()
    g = g.to(device)
    g.set_compute_dtype(torch.float32 if precision == "fp32" else torch.bfloat16)
    return m, g


def make_batch(seed, B, T_src, T_mel, device):
    from visual_onoma_to_wave_amd import synth
    b = synth.acoustic_batch(seed, B, T_src, T_mel)
    t = {k: (torch.from_numpy(v).to(device) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    return (t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
            t["max_mel_len"], None, None, t["d_targets"], t["images"], None, True)


def step(model, gen, args):
    out = model(*args)
    return gen.run(out[1])  # postnet mel is already channels-last (B, T, 80): no transpose


def cpu_baseline(budget_s, T_src, T_mel):
    """The oracle (CPU fp32 restatement, parity-pinned to the reference) on a bounded
    sample of the same workload: B=1 utterances, end-to-end, timed on this host."""
    from helpers import hifigan_arrays, hifigan_h, stats, vtts_arrays
    from oracle import acoustic as A
    from oracle import vocoder as V
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    sd = A.complete_state_dict(vtts_arrays(), stats()["energy"])
    gsd = V.fold_weight_norm({k: torch.from_numpy(np.array(v)) for k, v in hifigan_arrays().items()})
    h = hifigan_h()
    args = make_batch(7, 1, T_src, T_mel, "cpu")
    n, t0 = 0, time.perf_counter()
    with torch.no_grad():
        while True:
            out = A.vtts_forward(sd, *args[:11], energy_stats=stats()["energy"])
            V.generator(gsd, out[1].transpose(1, 2), h)
            n += 1
            if time.perf_counter() - t0 >= budget_s or n >= 50:
                break
    dt = time.perf_counter() - t0
    samples = n * T_mel * HOP
    return {"value": samples / dt, "unit": "audio samples/s", "cores": threads, "kind": "port",
            "sample": f"{n} x (1 utterance: T_src={T_src}, T_mel={T_mel} -> {T_mel * HOP} samples), "
                      f"oracle fp32 torch-CPU, {dt:.1f} s",
            "x_realtime": samples / dt / SR}


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    if a.mode == "gan":
        if a.batch == 32:
            a.batch = 16  # scripts/hifigan/config.json batch_size
        bench_gan(a, dev, rank, world, dist)
        if dist:
            dist.destroy_process_group()
        return
    if a.mode == "train":
        bench_train(a, dev, rank, world, dist)
        if dist:
            dist.destroy_process_group()
        return

    model, gen = build_models(dev, a.precision)
    args = make_batch(1234 + rank, a.batch, a.src_len, a.mel_len, dev)
    with torch.no_grad():
        for _ in range(a.warmup):
            step(model, gen, args)
        torch.cuda.synchronize()

        from visual_onoma_to_wave_amd.profiling import KernelTimer
        tags = [f"mrf_s{i}" for i in range(4)]
        timer = KernelTimer(tags if not a.no_kernel_timer else [])
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with timer:
            for _ in range(a.steps):
                wav = step(model, gen, args)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    assert wav.shape == (a.batch, a.mel_len * HOP) and torch.isfinite(wav).all()
    samples = a.batch * a.mel_len * HOP * a.steps * world
    frames = a.batch * a.mel_len * a.steps * world
    value = samples / elapsed

    # dominant kernel: the MRF stage with the largest total time (HIP events, same stream)
    roof = None
    ks = timer.summary()
    if ks:
        tag, d = max(ks.items(), key=lambda kv: kv[1]["total_ms"])
        achieved = d["flops_per_launch"] / (d["avg_ms"] * 1e-3) / 1e12
        peak = F32_PEAK_TFLOPS if a.precision == "fp32" else BF16_PEAK_TFLOPS
        pmc = {}  # HBM bytes per launch from the committed rocprofv3 PMC passes (tools/pmc_round.sh)
        tf = os.path.join(REPO, "profiles", "traffic_r01.json")
        if os.path.exists(tf):
            with open(tf) as f:
                pmc = {k: v.get("hbm_bytes_per_launch") for k, v in json.load(f).items()}
        traffic = pmc.get(tag)
        roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4), "traffic": traffic,
                "kernel": f"{' + '.join(d['kernels'])} (HiFi-GAN MRF stage {tag[-1]})",
                "launches": d["launches"], "avg_launch_ms": round(d["avg_ms"], 4),
                "flops_per_launch": d["flops_per_launch"],
                "algorithmic_bytes_per_launch": d["bytes_per_launch"],
                "all_stages": {k: {"kernel": " + ".join(v["kernels"]), "avg_ms": round(v["avg_ms"], 4),
                                   "launches": v["launches"],
                                   "tflops": round(v["flops_per_launch"] / (v["avg_ms"] * 1e-3) / 1e12, 1),
                                   "hbm_gbs_algorithmic": round(v["bytes_per_launch"] / (v["avg_ms"] * 1e-3) / 1e9, 1),
                                   # measured HBM bytes (PMC) over this run's launch time: the
                                   # north star's "HBM roofline on the MRF" for the narrow stages
                                   "hbm_frac_pmc": (round(pmc[k] / (v["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 3)
                                                    if pmc.get(k) else None)}
                               for k, v in sorted(ks.items())}}

    cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu = cpu_baseline(a.cpu_seconds, a.src_len, a.mel_len)

    if rank == 0:
        line = {
            "metric": "end-to-end audio samples/sec (22.05 kHz) + mel-frames/sec, batch 32, 1->8 GPU",
            "value": round(value, 1), "unit": "audio samples/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": {"mixed": "bf16 (encoder+variance adaptor fp32)", "bf16": "bf16", "fp32": "f32"}[a.precision],
            "data": "synthetic (procedural glyph strips, seeded durations; deterministic random weights)",
            "config": {"workload": "C2+C3 end-to-end: vTTS (B, T_src=12, teacher-forced T_mel=512, predicted "
                                   "energy) -> HiFi-GAN V1 generator -> B x 131072 samples",
                       "model": "vTTS (35.3M) + HiFi-GAN V1 (13.9M)", "global_batch": a.batch * world,
                       "per_gpu_batch": a.batch, "seq_len": a.mel_len, "src_len": a.src_len,
                       "parallelism": f"replicas x{world} (no data-path collective)"},
            "mel_frames_per_s": round(frames / elapsed, 1),
            "x_realtime": round(value / SR, 1),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
