"""Live per-kernel timing with HIP events on the launching stream.

``ops.conv1d(..., tag=...)`` brackets its launch with a pair of events when a
``KernelTimer`` watching that tag is installed, so bench.py can report the dominant
kernel's average launch duration (and algorithmic FLOP/s) over its own timed region,
on the stream the kernel actually runs on.

``KernelTimer.group(tag)`` brackets a run of consecutive launches of one tag (an MRF stage:
its 7 ResBlock launches, nothing else in between) with ONE event pair instead of a pair per
launch: the per-launch average is the run's elapsed time over its launch count, and the
event packets no longer sit between every two launches of the timed step.
"""

import contextlib

import torch

_GROUPED = object()  # start() token for launches inside an open group

_ACTIVE = None


class KernelTimer:
    def __init__(self, tags):
        self.tags = set(tags)
        self.pending = []  # (tag, start_event, end_event, flops, bytes, kernel label)
        self.groups = []   # (tag, start_event, end_event, launches, flops, bytes, kernel labels)
        self._grp = None

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
        if self._grp is not None:
            return _GROUPED
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def stop(self, tag, start_ev, flops, nbytes, kernel=None):
        if start_ev is _GROUPED:
            g = self._grp
            if tag != g["tag"]:
                raise RuntimeError(f"KernelTimer: launch tagged {tag} inside the {g['tag']} group")
            g["launches"] += 1
            g["flops"] += flops
            g["bytes"] += nbytes
            if kernel and kernel not in g["kernels"]:
                g["kernels"].append(kernel)
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.pending.append((tag, start_ev, ev, flops, nbytes, kernel))

    @contextlib.contextmanager
    def group(self, tag):
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        self._grp = dict(tag=tag, launches=0, flops=0.0, bytes=0.0, kernels=[])
        try:
            yield
        finally:
            g, self._grp = self._grp, None
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            if g["launches"]:
                self.groups.append((tag, s, e, g["launches"], g["flops"], g["bytes"], g["kernels"]))

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
        for tag, s, e, n, fl, nb, kerns in self.groups:
            d = out.setdefault(tag, dict(launches=0, total_ms=0.0, flops=0.0, bytes=0.0, kernels=[]))
            d["kernels"] += [k for k in kerns if k not in d["kernels"]]
            d["launches"] += n
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
