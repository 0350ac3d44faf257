"""Two-stage synthesis pipeline for serving on one GPU: glyph strips -> mel (vTTS) -> waveform
(HiFi-GAN), with the acoustic model of batch i + 1 on its own stream while the vocoder of batch i
runs on the caller's stream.

The acoustic model (``scripts/model/vtts.py:47-119``) is a chain of small, latency-bound kernels
at T_src = 12 / T_mel = 512 (2 ms for B = 32 alone, far from filling 256 CUs); the vocoder
(``scripts/hifigan/models.py:149-165``) fills the chip.  Overlapping them hides part of the
former behind the latter (bench.py: 13.67 -> 13.06 ms per B = 32 step).

Stream ordering.  ``submit`` first makes the acoustic stream wait for the caller's stream, so
inputs the caller produced there just before (``utils.tools.to_device`` lays glyph batches out
with a kernel on the current stream) are complete before the model reads them, and records every
CUDA input on the acoustic stream, so the caching allocator does not hand an input's memory out
while the acoustic model still reads it, even if the caller drops it right after ``submit``.
Each submitted batch's mel reaches the vocoder through an event; its memory is recorded on the
vocoder stream likewise.
"""

import collections

import torch


class SynthesisPipeline:
    """``submit(*model_args)`` starts the acoustic model of a batch; ``next_wav()`` vocodes the
    oldest submitted batch on the current stream and returns (acoustic outputs, wav (B, N))."""

    def __init__(self, model, vocoder, device=None):
        self.model, self.vocoder = model, vocoder
        self.device = torch.device(device) if device is not None else next(vocoder.parameters()).device
        self.acoustic_stream = torch.cuda.Stream(self.device)
        self._pending = collections.deque()

    def submit(self, *model_args):
        caller = torch.cuda.current_stream(self.device)
        self.acoustic_stream.wait_stream(caller)
        for a in model_args:
            if torch.is_tensor(a) and a.is_cuda:
                a.record_stream(self.acoustic_stream)
        with torch.cuda.stream(self.acoustic_stream):
            out = self.model(*model_args)
            ev = torch.cuda.Event()
            ev.record(self.acoustic_stream)
        self._pending.append((out, ev))

    def pending(self):
        return len(self._pending)

    def next_wav(self):
        if not self._pending:
            raise RuntimeError("SynthesisPipeline.next_wav: nothing submitted")
        out, ev = self._pending.popleft()
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(ev)
        for t in out:
            if torch.is_tensor(t) and t.is_cuda:
                t.record_stream(cur)
        return out, self.vocoder.run(out[1])  # postnet mel is channels-last (B, T, 80): no transpose
