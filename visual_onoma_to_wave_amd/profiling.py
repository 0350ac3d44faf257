"""Live per-kernel timing with HIP events on the launching stream.

``ops.conv1d(..., tag=...)`` brackets its launch with a pair of events when a
``KernelTimer`` watching that tag is installed, so bench.py can report the dominant
kernel's average launch duration (and algorithmic FLOP/s) over its own timed region,
on the stream the kernel actually runs on.
"""

import torch

_ACTIVE = None


class KernelTimer:
    def __init__(self, tags):
        self.tags = set(tags)
        self.pending = []  # (tag, start_event, end_event, flops, bytes, kernel label)

    def __enter__(self):
        global _ACTIVE
        _ACTIVE = self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = None

    def watching(self, tag):
        return tag in self.tags

    def start(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, tag, start_ev, flops, nbytes, kernel=None):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.pending.append((tag, start_ev, ev, flops, nbytes, kernel))

    def summary(self):
        """{tag: dict(launches, avg_ms, flops_per_launch, bytes_per_launch, kernels)} (synchronizes)."""
        torch.cuda.synchronize()
        out = {}
        for tag, s, e, fl, nb, kern in self.pending:
            d = out.setdefault(tag, dict(launches=0, total_ms=0.0, flops=0.0, bytes=0.0, kernels=[]))
            if kern and kern not in d["kernels"]:
                d["kernels"].append(kern)
            d["launches"] += 1
            d["total_ms"] += s.elapsed_time(e)
            d["flops"] += fl
            d["bytes"] += nb
        for d in out.values():
            n = d["launches"]
            d["avg_ms"] = d["total_ms"] / n
            d["flops_per_launch"] = d["flops"] / n
            d["bytes_per_launch"] = d["bytes"] / n
        return out


def active():
    return _ACTIVE
