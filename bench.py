#!/usr/bin/env python3
"""End-to-end visual-onomatopoeia -> 22.05 kHz waveform throughput on MI355X.

Headline (``--mode infer``, the default): one step = one batch of B synthetic rendered-glyph
strips (B x 1 x 24 x 102*T_src, T_src=12) through the acoustic model (teacher-forced durations
summing to T_mel=512 frames, predicted energy) and the HiFi-GAN V1
generator on its postnet mel (config C3 shape per utterance) -> B x 131,072 samples.  The same
run also measures BASELINE.json's per-config lines C2 (acoustic only, B=32, mel-frames/s),
C3 (generator only, B=64 x 80 x 512, samples/s) and -- on one GPU -- C4 (the acoustic training
step, B=32 x 512 frames) and C5 (the HiFi-GAN V1 training step, B=16 x 8192 samples) as graphed
single-GPU steps, each with its own roofline, under ``configs`` of the one JSON line.  Inputs are resident in HBM before every timed region.
Multi-GPU: one process per GPU (torchrun), every rank synthesises its own batch (utterances
are independent: replicas, no data-path collective), only the timing uses a
barrier and a MAX all-reduce.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch 32] [--precision mixed]
                    [--mode infer|c2|c3|train|gan] [--comm-dtype fp32|bf16]

Prints ONE JSON line (rank 0) with the metric of BASELINE.json, the dominant kernel's
roofline (HIP events on the launching stream over the timed region) and the CPU baseline
(the oracle restatement timed on this host: BASELINE.md's C1 / C2 / C3 plan).
"""

import argparse
import json
import os
import platform
import sys
import time

# before the HIP runtime initialises (graphed training steps, visual_onoma_to_wave_amd/train.py)
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

import numpy as np  # noqa: E402
import torch  # noqa: E402

REPO = os.path.dirname(os.path.abspath(__file__))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

SR = 22050
HOP = 256
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
BF16_PEAK_TFLOPS = 2500.0      # dense bf16 MFMA (no sparsity)
F32_PEAK_TFLOPS = 157.3
TRAFFIC_FILE = os.path.join("profiles", "traffic_r06.json")  # committed rocprofv3 PMC passes (tools/pmc_round.sh)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (default 32; c3: 64; gan: 16)")
    ap.add_argument("--src-len", type=int, default=12)
    ap.add_argument("--mel-len", type=int, default=512)
    ap.add_argument("--precision", default="mixed", choices=["mixed", "bf16", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="CPU-baseline budget (0 = skip)")
    ap.add_argument("--no-kernel-timer", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="infer: skip the C2 / C3 / C4 / C5 sub-measurements")
    ap.add_argument("--no-train-configs", action="store_true", help="infer: skip the C4 / C5 sub-measurements")
    ap.add_argument("--no-graph", action="store_true",
                    help="c2 (also inside infer) / train / gan: eager calls instead of one HIP graph")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="infer: run acoustic model and vocoder back to back instead of overlapping the acoustic "
                         "model of batch i+1 (own stream) with the vocoder of batch i")
    ap.add_argument("--stft-loss", type=float, default=0.0,
                    help="gan: weight of the auxiliary multi-resolution STFT loss (0 = HiFi-GAN V1 losses only)")
    ap.add_argument("--comm-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="train / gan under torchrun: gradient all-reduce dtype")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: every rank joins a gloo group, the ranks are "
                         "all-gathered and rank 0 prints them (no model, no CUDA call)")
    ap.add_argument("--mode", default="infer", choices=["infer", "c2", "c3", "train", "gan"],
                    help="infer: end-to-end synthesis (headline, with C2 / C3 sub-lines); c2: acoustic model "
                         "only; c3: HiFi-GAN generator only (B=64); train: C4 training step (DDP); "
                         "gan: C5 HiFi-GAN training step (DDP)")
    a = ap.parse_args()
    if a.batch is None:
        a.batch = {"c3": 64, "gan": 16}.get(a.mode, 32)  # gan: scripts/hifigan/config.json batch_size
    return a


# ----------------------------------------------------------------------------------- timing helpers

def timed(fn, steps, dist):
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed, out


def _pmc_traffic():
    tf = os.path.join(REPO, TRAFFIC_FILE)
    if not os.path.exists(tf):
        return {}
    with open(tf) as f:
        return {k: v.get("hbm_bytes_per_launch") for k, v in json.load(f).items()}


def roofline(ks, peak, label, batch=32):
    """Dominant tagged kernel (largest total time) -> the roofline object of the bench line.
    The committed PMC traffic was measured at B = 32 per launch; per-launch bytes scale with B."""
    if not ks:
        return None
    tag, d = max(ks.items(), key=lambda kv: kv[1]["total_ms"])
    achieved = d["flops_per_launch"] / (d["avg_ms"] * 1e-3) / 1e12
    pmc = {k: (v * batch / 32.0 if v else v) for k, v in _pmc_traffic().items()}
    stages = {}
    for k, v in sorted(ks.items()):
        stages[k] = {"kernel": " + ".join(v["kernels"]), "avg_ms": round(v["avg_ms"], 4), "launches": v["launches"],
                     "tflops": round(v["flops_per_launch"] / (v["avg_ms"] * 1e-3) / 1e12, 1),
                     "mfma_frac": round(v["flops_per_launch"] / (v["avg_ms"] * 1e-3) / 1e12 / peak, 3),
                     "hbm_gbs_algorithmic": round(v["bytes_per_launch"] / (v["avg_ms"] * 1e-3) / 1e9, 1),
                     # algorithmic bytes (read x + acc once, write y once, weights once) over the launch
                     # time: the fraction of the HBM roofline the stage would reach at zero wasted traffic
                     "hbm_frac_algorithmic": round(v["bytes_per_launch"] / (v["avg_ms"] * 1e-3) / 1e9
                                                   / HBM_PEAK_GBS, 3),
                     # measured HBM bytes (committed PMC passes) over this run's launch time: the north
                     # star's "HBM roofline on the MRF" for the narrow stages
                     "hbm_frac_pmc": (round(pmc[k] / (v["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 3)
                                      if pmc.get(k) else None)}
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": pmc.get(tag),
            "traffic_source": (f"{TRAFFIC_FILE} (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes, committed; "
                               "not measured in this run)") if pmc.get(tag) else None,
            "kernel": f"{' + '.join(d['kernels'])} ({label(tag)})", "tag": tag,
            "launches": d["launches"], "avg_launch_ms": round(d["avg_ms"], 4),
            "flops_per_launch": d["flops_per_launch"], "algorithmic_bytes_per_launch": d["bytes_per_launch"],
            "all_stages": stages}


def _mrf_label(tag):
    return f"HiFi-GAN MRF stage {tag[-1]}" if tag.startswith("mrf_s") else tag


# ----------------------------------------------------------------------------------- models / inputs

def build_models(device, precision, acoustic=True, vocoder=True):
    from helpers import configs, hifigan_arrays, hifigan_h, vtts_arrays
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.model import vTTS
    m = g = None
    if acoustic:
        m = vTTS(*configs())
        load_into(m, vtts_arrays())
        m = m.to(device).eval().set_precision(precision)
    if vocoder:
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


def make_mels(seed, B, T, device):
    """C3 input: mel = clamp(N(-5, 2), -11.513, 2.5)."""
    gen = torch.Generator().manual_seed(seed)
    return (torch.randn(B, 80, T, generator=gen) * 2 - 5).clamp(-11.513, 2.5).to(device)


# ----------------------------------------------------------------------------------- CPU baseline

def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(budget_s, T_src, T_mel, B_headline):
    """BASELINE.md's plan on the oracle (CPU fp32 restatement, parity-pinned to the reference):
    C1 single utterance x real time, the full C2 acoustic batch, C3 at B = 4; the headline value
    is the end-to-end rate of a B_headline batch composed from the C2 and C3 rates."""
    from helpers import hifigan_arrays, hifigan_h, stats, vtts_arrays
    from oracle import acoustic as A
    from oracle import vocoder as V
    threads = min(16, os.cpu_count() or 1)  # the GPU box's CPU share is 16 (os.cpu_count() is the host's)
    torch.set_num_threads(threads)
    sd = A.complete_state_dict(vtts_arrays(), stats()["energy"])
    gsd = V.fold_weight_norm({k: torch.from_numpy(np.array(v)) for k, v in hifigan_arrays().items()})
    h = hifigan_h()
    es = stats()["energy"]

    def rep(fn, share):
        n, t0 = 0, time.perf_counter()
        while True:
            fn()
            n += 1
            if time.perf_counter() - t0 >= share * budget_s or n >= 20:
                break
        return (time.perf_counter() - t0) / n, n

    with torch.no_grad():
        c1 = make_batch(1234, 1, 4, 50, "cpu")
        t_c1, n1 = rep(lambda: V.generator(gsd, A.vtts_forward(sd, *c1[:11], energy_stats=es)[1].transpose(1, 2), h),
                       0.15)
        c2 = make_batch(1234, 32, T_src, T_mel, "cpu")
        t_c2, n2 = rep(lambda: A.vtts_forward(sd, *c2[:11], energy_stats=es), 0.35)
        mel4 = make_mels(1234, 4, T_mel, "cpu")
        t_c3, n3 = rep(lambda: V.generator(gsd, mel4, h), 0.5)
    c1_samples = 50 * HOP
    c3_rate = 4 * T_mel * HOP / t_c3
    t_e2e = t_c2 * B_headline / 32 + B_headline * T_mel * HOP / c3_rate
    value = B_headline * T_mel * HOP / t_e2e
    return {"value": value, "unit": "audio samples/s", "cores": threads, "kind": "port",
            "host_cpu_count": os.cpu_count(), "threads": threads, "cpu_model": cpu_model(),
            "sample": (f"oracle fp32 torch-CPU, {threads} threads: C1 {n1} x (B=1, T_src=4, T_mel=50), C2 {n2} x "
                       f"(B=32, T_src={T_src}, T_mel={T_mel}), C3 {n3} x (B=4 x 80 x {T_mel}); value = "
                       f"B={B_headline} end to end composed from the C2 and C3 rates"),
            "x_realtime": value / SR,
            "c1_x_realtime": c1_samples / t_c1 / SR, "c1_ms": round(t_c1 * 1e3, 2),
            "c2_mel_frames_per_s": 32 * T_mel / t_c2, "c2_ms": round(t_c2 * 1e3, 1),
            "c3_samples_per_s": c3_rate, "c3_ms_b4": round(t_c3 * 1e3, 1)}


# ----------------------------------------------------------------------------------- inference configs

def measure_c2(a, dev, dist, model=None):
    """C2: acoustic forward, B=32 synthetic glyph batch, teacher-forced T_mel=512 (mel-frames/s);
    roofline on the decoder FFN's k=9 conv (the largest share of the 771 GFLOP batch)."""
    from visual_onoma_to_wave_amd.profiling import KernelTimer
    rank = int(os.environ.get("RANK", "0"))
    if model is None:
        model, _ = build_models(dev, a.precision, vocoder=False)
    B = 32 if a.mode != "c2" else a.batch
    args = make_batch(1234 + rank, B, a.src_len, a.mel_len, dev)
    with torch.no_grad():
        for _ in range(a.warmup):
            model(*args)
        # the teacher-forced forward has static shapes and no host synchronisation: it is captured once
        # as a HIP graph and the timed region replays it (--no-graph: eager calls)
        graph, hip_graph = None, False
        if not a.no_graph:
            try:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    model(*args)
                torch.cuda.current_stream().wait_stream(s)
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph):
                    gout = model(*args)
                hip_graph = True
            except RuntimeError as e:  # report, and time the eager forward instead -- on a fresh state
                print(f"[bench] C2 graph capture failed ({e}); timing eager calls", file=sys.stderr)
                graph = None
                torch.cuda.synchronize()
                for _ in range(max(a.warmup, 1)):  # re-warm the allocator / packs outside any capture
                    model(*args)
                torch.cuda.synchronize()
        if graph is not None:
            elapsed, _ = timed(graph.replay, a.steps, dist)
            out = gout
        else:
            elapsed, out = timed(lambda: model(*args), a.steps, dist)
        # roofline pass: HIP events around each decoder FFN w_1 launch, outside the timed region
        timer = KernelTimer(["dec_ffn_w1"] if not a.no_kernel_timer else [])
        with timer:
            timed(lambda: model(*args), a.steps, dist)
    assert torch.isfinite(out[1]).all()
    world = dist.get_world_size() if dist else 1
    frames = B * a.mel_len * a.steps * world
    peak = F32_PEAK_TFLOPS if a.precision == "fp32" else BF16_PEAK_TFLOPS
    return {"metric": "C2 acoustic forward mel-frames/sec (vTTS, batch 32, teacher-forced T_mel=512)",
            "value": round(frames / elapsed, 1), "unit": "mel-frames/s", "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "per_gpu_batch": B, "tflops_step": round(771.4e9 * B / 32 / (elapsed / a.steps) / 1e12, 1),
            "hip_graph": hip_graph,
            # rounds <= 4 timed eager forwards; from round 5 the timed region replays one HIP graph
            "timing_mode": "hip_graph_replay" if hip_graph else "eager",
            "roofline": dict(roofline(timer.summary(), peak, lambda t: "decoder FFN w_1 conv, k=9 256->1024"),
                             measured_in="separate eager pass with an event pair per w_1 launch (not the timed region)")}


def measure_c3(a, dev, dist, gen=None):
    """C3: HiFi-GAN generator on B=64 x 80 x 512 mels (samples/s); roofline on the MRF stage
    with the largest total time."""
    from visual_onoma_to_wave_amd.profiling import KernelTimer
    rank = int(os.environ.get("RANK", "0"))
    if gen is None:
        _, gen = build_models(dev, a.precision, acoustic=False)
    B = 64 if a.mode != "c3" else a.batch
    mel = make_mels(1234 + rank, B, a.mel_len, dev)
    from visual_onoma_to_wave_amd.hifigan import models as hm
    with torch.no_grad():
        for _ in range(a.warmup):
            gen(mel)
        elapsed, wav = timed(lambda: gen(mel), a.steps, dist)
        # roofline pass with per-stage events, MRF chains serialized (see infer)
        timer = KernelTimer([f"mrf_s{i}" for i in range(4)] if not a.no_kernel_timer else [])
        streams, hm.MRF_STREAMS = hm.MRF_STREAMS, False
        try:
            gen(mel)
            with timer:
                timed(lambda: gen(mel), a.steps, dist)
        finally:
            hm.MRF_STREAMS = streams
    assert wav.shape == (B, 1, a.mel_len * HOP) and torch.isfinite(wav).all()
    world = dist.get_world_size() if dist else 1
    samples = B * a.mel_len * HOP * a.steps * world
    peak = F32_PEAK_TFLOPS if a.precision == "fp32" else BF16_PEAK_TFLOPS
    return {"metric": "C3 HiFi-GAN generator audio samples/sec (batch 64 x 80-mel x 512-frame)",
            "value": round(samples / elapsed, 1), "unit": "audio samples/s",
            "ms_per_step": round(elapsed / a.steps * 1e3, 3), "per_gpu_batch": B,
            "x_realtime": round(samples / elapsed / SR, 1),
            "tflops_step": round(2398848.0 * B * a.mel_len * HOP / (elapsed / a.steps) / 1e12, 1),
            "roofline": roofline(timer.summary(), peak, _mrf_label, batch=B)}


# ----------------------------------------------------------------------------------- training configs

C4_FWD_FLOPS_B32 = 771.4e9    # vTTS forward at B = 32, T_src = 12, T_mel = 512
GEN_FLOPS_PER_SAMPLE = 2398848.0  # HiFi-GAN V1 generator FLOPs per output sample
MSD_CFG = [(1, 128, 15, 1, 1, 7), (128, 128, 41, 2, 4, 20), (128, 256, 41, 2, 16, 20), (256, 512, 41, 4, 16, 20),
           (512, 1024, 41, 4, 16, 20), (1024, 1024, 41, 1, 16, 20), (1024, 1024, 5, 1, 1, 2)]
# dominant kernel and kernel families (time, FLOPs, fraction of peak) of the training steps in the
# committed serialized kernel traces (tools/train_prof.sh -> tools/train_dominant.py)
TRAIN_DOMINANT = os.path.join("profiles", "r06", "train_dominant.json")


def disc_forward_flops(T, B):
    """Algorithmic FLOPs of one MPD + MSD forward (HiFi-GAN V1) on B waveforms of T samples."""
    tot = 0
    ch = [1, 32, 128, 512, 1024, 1024]
    for p in (2, 3, 5, 7, 11):
        H = -(-T // p)
        for i in range(5):
            Ho = (H + 4 - 5) // (3 if i < 4 else 1) + 1
            tot += 2 * ch[i] * ch[i + 1] * 5 * Ho * p * B
            H = Ho
        tot += 2 * 1024 * 3 * H * p * B
    L0 = T
    for sc in range(3):
        if sc:
            L0 = (L0 + 4 - 4) // 2 + 1  # AvgPool1d(4, 2, padding=2)
        L = L0
        for ci, co, k, s_, g, p in MSD_CFG:
            L = (L + 2 * p - k) // s_ + 1
            tot += 2 * (ci // g) * co * k * L * B
        tot += 2 * 1024 * 3 * L * B
    return float(tot)


def train_step_flops(mode, B, seg=8192):
    """Algorithmic FLOPs of one training step (forward counts x the backward's 2 passes):
    C4: 3 x the vTTS forward; C5: the generator 3 x (forward, input and weight gradients), the
    D step 3 x D(real + fake), the G step D(fake) + D(real features) + D's input gradient."""
    if mode == "train":
        return 3 * C4_FWD_FLOPS_B32 * B / 32
    return 3 * GEN_FLOPS_PER_SAMPLE * B * seg + 9 * disc_forward_flops(seg, B)


def _dominant(mode):
    try:
        with open(os.path.join(REPO, TRAIN_DOMINANT)) as f:
            return json.load(f).get(mode)
    except OSError:
        return None


def train_roofline(mode, B, ms, peak):
    fl = train_step_flops(mode, B)
    r = {"bound": "mfma", "achieved": round(fl / (ms * 1e-3) / 1e12, 2), "peak": peak, "unit": "TFLOP/s",
         "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4), "traffic": None,
         "flops_per_step": fl, "flops_source": "bench.train_step_flops (DESIGN.md section 7)",
         "measured_in": "whole graphed step (HIP-graph replays, wall clock over the timed steps)"}
    dom = _dominant(mode)
    if dom:  # from the committed serialized kernel trace of this step (not measured in this run)
        r["dominant_kernel"] = dom
    return r


def run_train(a, dev, rank, world, dist, B=None):
    """C4: scripts/04_train.py step (teacher-forced forward, FastSpeech2Loss, backward with the
    bucketed RCCL all-reduce, clip 1.0, Adam + schedule) on B utterances per GPU, replayed as
    one HIP graph (the all-reduces captured on the side-stream branch) unless --no-graph."""
    from helpers import configs, vtts_arrays
    from weights import load_into
    from visual_onoma_to_wave_amd import synth
    from visual_onoma_to_wave_amd.model import FastSpeech2Loss, ScheduledOptim, vTTS
    from visual_onoma_to_wave_amd.train import GradBucketer, GraphedTrainStep, train_step, unused_on_path
    B = B or a.batch
    pc, mc, tc = configs()
    m = vTTS(pc, mc, tc)
    load_into(m, vtts_arrays())
    m = m.to(dev).train().set_precision(a.precision)
    graphed = not a.no_graph
    opt = ScheduledOptim(m, tc, mc, 0, capturable=graphed)
    bk = None
    comm = torch.bfloat16 if a.comm_dtype == "bf16" else None
    if dist:
        skip = unused_on_path(m)
        bk = GradBucketer([p for p in m.parameters() if id(p) not in skip], comm_dtype=comm)
        bk.broadcast_parameters(m)
    b = synth.acoustic_batch(1234 + rank, B, a.src_len, a.mel_len)
    t = {k: (torch.from_numpy(v).to(dev) if isinstance(v, np.ndarray) else v) for k, v in b.items()}
    batch = (None, t["audiotypes"], t["texts"], t["src_lens"], t["max_src_len"], t["mels"], t["mel_lens"],
             t["max_mel_len"], t["e_targets"], None, t["d_targets"], t["images"], None)
    loss_fn = FastSpeech2Loss()
    if graphed:
        run = GraphedTrainStep(m, opt, loss_fn, bucketer=bk)
    else:
        def run(bt):
            return train_step(m, opt, loss_fn, bt, bucketer=bk)
    for _ in range(a.warmup):
        run(batch)
    elapsed, losses = timed(lambda: run(batch), a.steps, dist)
    frames = B * a.mel_len * a.steps * world
    n_grad = sum(p.numel() for p in (bk.params if bk else []))
    ms = elapsed / a.steps * 1e3
    peak = F32_PEAK_TFLOPS if a.precision == "fp32" else BF16_PEAK_TFLOPS
    return {
        "metric": "C4 training mel-frames/sec (FastSpeech2 + variance loss, DDP)", "value": round(frames / elapsed, 1),
        "unit": "mel-frames/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": a.precision, "data": "synthetic",
        "final_loss": round(float(losses[0].detach()) if torch.is_tensor(losses[0]) else float(losses[0]), 5),
        "hip_graph": graphed,
        "allreduce_bytes_per_step": n_grad * (2 if comm is not None else 4) if dist else 0,
        "roofline": train_roofline("train", B, ms, peak),
        "config": {"workload": "C4 train step", "per_gpu_batch": B, "global_batch": B * world,
                   "seq_len": a.mel_len, "src_len": a.src_len,
                   "parallelism": f"dp{world} (RCCL bucketed all-reduce, {a.comm_dtype})"}}


def run_gan(a, dev, rank, world, dist, B=None):
    """C5: HiFi-GAN V1 training step (generator + MPD + MSD, D step then G step with adversarial,
    feature-matching and 45 x mel-L1 losses, AdamW) on B segments of 8192 samples per GPU
    (scripts/hifigan/config.json: batch 16, segment 8192)."""
    from helpers import hifigan_arrays, hifigan_h
    from weights import load_into
    from visual_onoma_to_wave_amd import hifigan
    from visual_onoma_to_wave_amd.hifigan.discriminators import MelLoss
    B = B or a.batch
    h = hifigan.AttrDict(hifigan_h())
    g = hifigan.Generator(h)
    load_into(g, hifigan_arrays())
    g = g.to(dev)
    torch.manual_seed(1234)  # identical discriminator init on every rank (broadcast anyway)
    graphed = not a.no_graph
    tr = hifigan.HifiGanTrainer(g, h, distributed=dist is not None, device=dev, graphed=graphed,
                                comm_dtype=torch.bfloat16 if a.comm_dtype == "bf16" else None,
                                stft_loss_weight=a.stft_loss)
    run = tr.step_graphed if graphed else tr.step
    tr.set_compute_dtype(torch.float32 if a.precision == "fp32" else torch.bfloat16)
    seg = h.segment_size
    gen = torch.Generator().manual_seed(99 + rank)
    t = torch.arange(seg, dtype=torch.float32) / h.sampling_rate
    f0 = 110.0 + 330.0 * torch.rand(B, 1, generator=gen)
    y = (0.3 * torch.sin(2 * np.pi * f0 * t) + 0.05 * torch.randn(B, seg, generator=gen)).to(dev)
    with torch.no_grad():
        x = MelLoss(h.n_fft, h.num_mels, h.sampling_rate, h.hop_size, h.win_size, h.fmin, h.fmax).to(dev).mel(y)
    x = x.transpose(1, 2).contiguous()  # (B, 32, 80) channels-last generator input
    for _ in range(a.warmup):
        run(x, y)
    elapsed, losses = timed(lambda: run(x, y), a.steps, dist)
    samples = B * seg * a.steps * world
    ms = elapsed / a.steps * 1e3
    peak = F32_PEAK_TFLOPS if a.precision == "fp32" else BF16_PEAK_TFLOPS
    return {
        "metric": "C5 HiFi-GAN training audio samples/sec (G + MPD + MSD, DDP)", "value": round(samples / elapsed, 1),
        "unit": "audio samples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16" if a.precision != "fp32" else "f32",
        "data": "synthetic (sinusoid + noise segments, their mel as generator input)",
        "losses": {k: round(float(v), 4) for k, v in losses.items()},
        "hip_graph": graphed,
        "roofline": train_roofline("gan", B, ms, peak) if not a.stft_loss else None,
        "config": {"workload": "C5 HiFi-GAN V1 train step" + (
                       f" + {a.stft_loss} x multi-resolution STFT loss" if a.stft_loss else ""),
                   "per_gpu_batch": B, "global_batch": B * world,
                   "segment": seg, "parallelism": f"dp{world} (RCCL bucketed all-reduce, G and D, {a.comm_dtype})"}}


def bench_train(a, dev, rank, world, dist):
    res = run_train(a, dev, rank, world, dist)
    if rank == 0:
        res["ranks_seen"] = a.ranks_seen
        print(json.dumps(res))


def bench_gan(a, dev, rank, world, dist):
    res = run_gan(a, dev, rank, world, dist)
    if rank == 0:
        res["ranks_seen"] = a.ranks_seen
        print(json.dumps(res))


# ----------------------------------------------------------------------------------- launch

def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """``--gpus N`` without a torchrun environment: start N rank processes of this script (one
    per GPU, LOCAL_RANK = rank, rendezvous on 127.0.0.1) and exit with the worst exit code.
    Runs before anything touches the GPU; the ranks are children, never an exec of this
    process.  Rank 0's stdout carries the JSON line."""
    import signal
    import subprocess
    if "--dry-run" not in sys.argv:
        n_dev = torch.cuda.device_count()  # does not initialise the HIP runtime on this image
        if n > n_dev:
            sys.exit(f"bench.py: --gpus {n} but only {n_dev} GPU(s) visible")
    env = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = []
    for r in range(n):
        env_r = dict(env, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env_r))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    for q in pending:          # one rank failed: the others would hang in a collective
                        q.send_signal(signal.SIGTERM)
            time.sleep(0.05)
    except KeyboardInterrupt:
        for p in procs:
            p.send_signal(signal.SIGTERM)
        raise
    return rc


def rank_census(dist, world, rank, local, dev):
    """All-gather (rank, local_rank) of every process: the ranks the collective layer saw."""
    if dist is None:
        return [0]
    t = torch.tensor([rank, local], dtype=torch.int64, device=dev)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [int(p[0]) for p in parts]


def dry_run(a):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    try:
        seen = rank_census(dist, world, rank, local, "cpu")
        if rank == 0:
            print(json.dumps({"dry_run": True, "mode": a.mode, "gpus_requested": a.gpus,
                              "n_gpus": dist.get_world_size() if dist else 1, "ranks_seen": seen}))
    finally:
        if dist:
            dist.destroy_process_group()


# ----------------------------------------------------------------------------------- main

def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a.gpus))
    if a.dry_run:
        return dry_run(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
        world = dist.get_world_size()
    a.ranks_seen = rank_census(dist, world, rank, local, dev)

    try:
        if a.mode == "gan":
            bench_gan(a, dev, rank, world, dist)
        elif a.mode == "train":
            bench_train(a, dev, rank, world, dist)
        elif a.mode in ("c2", "c3"):
            res = (measure_c2 if a.mode == "c2" else measure_c3)(a, dev, dist)
            if rank == 0:
                res.update({"n_gpus": world, "ranks_seen": a.ranks_seen, "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
                            "scaling": "weak", "vs_baseline": None,
                            "dtype": {"mixed": "bf16 (encoder+variance adaptor fp32)", "bf16": "bf16",
                                      "fp32": "f32"}[a.precision] if a.mode == "c2" else
                            ("f32" if a.precision == "fp32" else "bf16"),
                            "data": "synthetic (deterministic random weights)",
                            "config": {"workload": a.mode.upper(), "per_gpu_batch": a.batch,
                                       "global_batch": a.batch * world, "seq_len": a.mel_len,
                                       "parallelism": f"replicas x{world} (no data-path collective)"}})
                print(json.dumps(res))
        else:
            infer(a, dev, rank, world, dist)
    finally:
        if dist:
            dist.destroy_process_group()


def infer(a, dev, rank, world, dist):
    from visual_onoma_to_wave_amd.hifigan import models as hm
    from visual_onoma_to_wave_amd.profiling import KernelTimer
    model, gen = build_models(dev, a.precision)
    args = make_batch(1234 + rank, a.batch, a.src_len, a.mel_len, dev)

    def seq_step():
        out = model(*args)
        return gen.run(out[1])  # postnet mel is already channels-last (B, T, 80): no transpose

    step = seq_step
    if not a.no_pipeline:
        # two-stage serving pipeline (visual_onoma_to_wave_amd.pipeline): the acoustic model of
        # batch i + 1 runs on its own stream while the vocoder synthesises batch i -- every step
        # still runs one whole acoustic pass and one whole vocoder pass
        from visual_onoma_to_wave_amd.pipeline import SynthesisPipeline
        pipe = SynthesisPipeline(model, gen, dev)

        def step():  # noqa: F811
            pipe.submit(*args)
            return pipe.next_wav()[1]

        with torch.no_grad():
            pipe.submit(*args)  # the pipeline's first stage, before the warm-up and timed steps

    with torch.no_grad():
        for _ in range(a.warmup):
            step()
        elapsed, wav = timed(step, a.steps, dist)  # the headline: no kernel timer in the timed region
        assert wav.shape == (a.batch, a.mel_len * HOP) and torch.isfinite(wav).all()
        # roofline pass: the same step run sequentially (acoustic model then vocoder on one stream, the
        # C = 256 MRF chains one after another), per-stage HIP events on the launching stream -- so
        # each kernel's duration is its own, as in the serialized rocprofv3 trace under profiles/
        timer = KernelTimer([f"mrf_s{i}" for i in range(4)] if not a.no_kernel_timer else [])
        streams, hm.MRF_STREAMS = hm.MRF_STREAMS, False
        try:
            seq_step()
            with timer:
                roof_elapsed, _ = timed(seq_step, a.steps, dist)
        finally:
            hm.MRF_STREAMS = streams
    samples = a.batch * a.mel_len * HOP * a.steps * world
    frames = a.batch * a.mel_len * a.steps * world
    value = samples / elapsed
    peak = F32_PEAK_TFLOPS if a.precision == "fp32" else BF16_PEAK_TFLOPS
    roof = roofline(timer.summary(), peak, _mrf_label, batch=a.batch)
    if roof is not None:
        roof["measured_in"] = (f"sequential roofline pass ({a.steps} steps, {roof_elapsed / a.steps * 1e3:.3f} ms per "
                               "step with events): no acoustic/vocoder overlap, MRF chains serialized")

    configs = None
    if not a.no_configs:  # BASELINE.json's per-config lines, same run, same models
        configs = {"C2": measure_c2(a, dev, dist, model), "C3": measure_c3(a, dev, dist, gen)}
        if world == 1 and not a.no_train_configs:
            # C4 / C5 as single-GPU graphed steps (BASELINE.json configs 4 and 5 at their per-GPU
            # batches; the DDP form is --mode train / gan under torchrun)
            configs["C4"] = run_train(a, dev, rank, world, dist, B=32)
            torch.cuda.empty_cache()
            configs["C5"] = run_gan(a, dev, rank, world, dist, B=16)

    cpu = None
    if rank == 0 and world == 1 and a.cpu_seconds > 0:
        cpu = cpu_baseline(a.cpu_seconds, a.src_len, a.mel_len, a.batch)

    if rank == 0:
        line = {
            "metric": "end-to-end audio samples/sec (22.05 kHz) + mel-frames/sec, batch 32, 1->8 GPU",
            "value": round(value, 1), "unit": "audio samples/s", "n_gpus": world, "ranks_seen": a.ranks_seen,
            "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": {"mixed": "bf16 (encoder+variance adaptor fp32)", "bf16": "bf16", "fp32": "f32"}[a.precision],
            "data": "synthetic (procedural glyph strips, seeded durations; deterministic random weights)",
            "config": {"workload": "C2+C3 end-to-end: vTTS (B, T_src=12, teacher-forced T_mel=512, predicted "
                                   "energy) -> HiFi-GAN V1 generator -> B x 131072 samples",
                       "model": "vTTS (35.3M) + HiFi-GAN V1 (13.9M)", "global_batch": a.batch * world,
                       "per_gpu_batch": a.batch, "seq_len": a.mel_len, "src_len": a.src_len,
                       "parallelism": f"replicas x{world} (no data-path collective)",
                       "pipeline": ("sequential" if a.no_pipeline else
                                    "acoustic(batch i+1) on its own stream || vocoder(batch i)")},
            "mel_frames_per_s": round(frames / elapsed, 1),
            "x_realtime": round(value / SR, 1),
            "roofline": roof,
            "configs": configs,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))


if __name__ == "__main__":
    main()
