"""Data-parallel training step (config C4; reference: scripts/04_train.py:115-175).

The reference trains with single-process ``nn.DataParallel`` (GPU0 broadcasts 141 MB of
parameters and reduce-adds 139 MB of gradients every step, 04_train.py:75).  Here: one
process per GPU (torchrun), parameters broadcast once, and a bucketed gradient all-reduce
over RCCL/xGMI launched from per-parameter post-accumulate hooks, so each bucket's
collective overlaps the rest of the backward on a separate stream.

Buckets are persistent flat buffers (~25 MB of fp32 gradients each: about 6 for the 139 MB
of the acoustic model).  When a bucket's last gradient has been accumulated its gradients
are gathered into the flat buffer by one multi-tensor copy on the compute stream (into a
bf16 copy of the bucket with ``comm_dtype=torch.bfloat16``: 69 MB per step on the wire), the
side stream all-reduces it in place (``ReduceOp.AVG`` on RCCL), and ``finish()`` points every
``p.grad`` at its slice of the averaged bucket -- no per-step ``torch.cat`` / copy-back, no
allocation.  Parameters that receive no gradient on the path (``encoder.src_word_emb`` with
image input, ``variance_adaptor.kurt_embedding`` without kurtosis conditioning) are left out.

The whole step -- forward, backward with the bucketed collectives, clipping and Adam -- is
capturable as one HIP graph (``GraphedTrainStep``), on one GPU and under torchrun (the RCCL
all-reduces are captured as graph nodes on the side-stream branch).

HIP graphs and this ROCm runtime: with the CLR's graph "packet capture" launch path (on by
default) replays of the C4 step computed wrong values -- losses read right after a replay
were stale and the second replay produced NaN even with a host wait in between
(tools/probes/graph_race_probe.py); the same graph launched through the ordinary node path
(``DEBUG_CLR_GRAPH_PACKET_CAPTURE=0``) replays 30 steps back to back with no host wait and
matches eager execution.  The package sets that variable at import (it is read when the HIP
runtime initialises, so import this package -- or export the variable -- before the first CUDA
call); ``GraphedTrainStep`` refuses to run when it is not in effect.
"""

import contextlib
import os

import torch
import torch.distributed as dist

from . import _base
from . import autograd as AG


def packet_capture_disabled():
    """True when the HIP runtime read DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 at its initialisation: the
    variable is "0" and it was not first set by this package after torch had initialised CUDA."""
    import visual_onoma_to_wave_amd as _pkg
    return os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0" and not _pkg.PACKET_CAPTURE_SET_LATE


class GradBucketer:
    """Bucketed, backward-overlapped gradient averaging across the default process group.

    ``comm_dtype``: dtype on the wire (None = the gradients' dtype, fp32; ``torch.bfloat16``
    halves the bytes, accumulation error ~4e-3 relative per element)."""

    def __init__(self, params, bucket_mb=25.0, group=None, comm_dtype=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.params = [p for p in params if p.requires_grad]
        # reverse registration order ~ the order gradients become ready in backward
        order = list(reversed(self.params))
        cap = int(bucket_mb * 1024 * 1024 / 4)
        self.buckets, cur, n = [], [], 0
        for p in order:
            if cur and n + p.numel() > cap:
                self.buckets.append(cur)
                cur, n = [], 0
            cur.append(p)
            n += p.numel()
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        dev = self.params[0].device if self.params else torch.device("cpu")
        self.flat, self.views, self.comm = [], [], []
        for b in self.buckets:
            dt = b[0].dtype
            if any(p.dtype != dt for p in b):
                raise TypeError("GradBucketer: one parameter dtype per bucket")
            flat = torch.zeros(sum(p.numel() for p in b), dtype=dt, device=dev)
            views, off = [], 0
            for p in b:
                views.append(flat[off: off + p.numel()].view_as(p))
                off += p.numel()
            self.flat.append(flat)
            self.views.append(views)
            self.comm.append(flat if comm_dtype in (None, dt) else torch.empty(flat.numel(), dtype=comm_dtype,
                                                                               device=dev))
        backend = dist.get_backend(group)
        self.avg = backend == "nccl"  # RCCL averages on the wire; gloo sums, then we scale
        self.side = torch.cuda.Stream(dev) if dev.type == "cuda" else None
        self.device = dev
        self.local_only = False      # warm-up before a capture: no collective at all
        self.capture_group = None    # the group the captured collectives run on (see capturing())
        self.hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]
        self.reset()

    @contextlib.contextmanager
    def warmup(self):
        """Steps run inside skip the collectives (each rank keeps its own gradients): the eager
        warm-up steps before a HIP-graph capture, whose updates ``TrainState`` undoes anyway.
        Everything else -- hooks, gathers into the buckets, the side stream -- runs as usual, so
        the warm-up still exercises the allocator and the pack caches the capture will use."""
        prev, self.local_only = self.local_only, True
        try:
            yield self
        finally:
            self.local_only = prev

    @contextlib.contextmanager
    def capturing(self):
        """Collectives issued inside go to a process group that only ever carries captured
        collectives (``graph_group``).  An eager collective still in the watchdog's list of
        in-flight works when a capture begins has its end event on its group's stream; if the
        capture joins that stream the watchdog's query of the event aborts the process
        ("operation not permitted on an event last recorded in a capturing stream").  The graph
        group never has an eager work, so no such race exists -- whatever the timing."""
        prev = self.capture_group
        self.capture_group = graph_group(self.group, self.device)
        try:
            yield self
        finally:
            self.capture_group = prev

    def reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.launched = [False] * len(self.buckets)

    def broadcast_parameters(self, module):
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, 0, group=self.group)

    def _gather(self, i):
        """Bucket i's gradients -> its comm buffer (one multi-tensor copy on the compute stream;
        a parameter that got no gradient this step contributes zeros)."""
        b, views = self.buckets[i], self.views[i]
        src, dst = [], []
        comm = self.comm[i]
        tgt = views if comm is self.flat[i] else None
        off = 0
        for p, v in zip(b, views):
            n = p.numel()
            d = v if tgt is not None else comm[off: off + n].view_as(p)
            off += n
            g = p.grad
            if g is None:
                d.zero_()
            elif g.data_ptr() != d.data_ptr():
                src.append(g)
                dst.append(d)
        if src:
            torch._foreach_copy_(dst, src)

    def _launch(self, i):
        self._gather(i)
        buf = self.comm[i]
        if self.side is not None:
            main = torch.cuda.current_stream(buf.device)
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                self._reduce(i, buf)
        else:
            self._reduce(i, buf)
        self.launched[i] = True

    def _reduce(self, i, buf):
        group = self.capture_group if self.capture_group is not None else self.group
        if self.local_only:
            pass
        elif self.avg:
            dist.all_reduce(buf, op=dist.ReduceOp.AVG, group=group)
        else:
            dist.all_reduce(buf, group=group)
            buf.div_(self.world)
        if buf is not self.flat[i]:
            self.flat[i].copy_(buf)

    def _ready(self, p):
        i = self.bucket_of[id(p)]
        self.pending[i] -= 1
        if self.pending[i] == 0:
            self._launch(i)

    def finish(self):
        """Launch the buckets that did not complete (parameters without a gradient this step),
        join the side stream and point every ``p.grad`` at its averaged bucket slice."""
        for i, done in enumerate(self.launched):
            if not done:
                self._launch(i)
        if self.side is not None:
            torch.cuda.current_stream(self.side.device).wait_stream(self.side)
        for b, views in zip(self.buckets, self.views):
            for p, v in zip(b, views):
                p.grad = v
        self.reset()


def unused_on_path(model):
    """Parameters the image-input, energy-only configuration never touches."""
    skip = set()
    if hasattr(model, "encoder"):
        skip.add(id(model.encoder.src_word_emb.weight))
    va = getattr(model, "variance_adaptor", None)
    if va is not None and not va.is_kurtosis:
        skip.add(id(va.kurt_embedding.weight))
    return skip


def train_step(model, optimizer, loss_fn, batch, grad_clip=1.0, bucketer=None, use_image=True):
    """One step of scripts/04_train.py:128-141: forward, loss, backward (with overlapped
    all-reduce), clip_grad_norm_(grad_clip), ScheduledOptim.step_and_update_lr, zero_grad."""
    output = model(*(batch[1:]), use_image)
    losses = loss_fn(batch, output)
    losses[0].backward()
    if bucketer is not None:
        bucketer.finish()
    params = [p for p in model.parameters() if p.grad is not None]
    torch.nn.utils.clip_grad_norm_(params, grad_clip)
    optimizer.step_and_update_lr()
    optimizer.zero_grad()
    return losses


class TrainState:
    """Snapshot / restore of a model's parameters and buffers and of optimizers' state, so eager
    warm-up steps before a HIP-graph capture leave no trace (each call of a graphed step applies
    exactly one update).  Optimizer state tensors are restored in place (the capture records
    their addresses); state created by the warm-up is reset to a fresh optimizer's (zeros)."""

    def __init__(self, modules, optimizers):
        self.tensors = []
        for m in modules:
            self.tensors += [t for t in list(m.parameters()) + list(m.buffers())]
        self.optimizers = optimizers
        with torch.no_grad():
            self.saved = [t.detach().clone() for t in self.tensors]
            self.state = [{id(p): {k: (v.clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                           for p, st in o.state.items()} for o in optimizers]

    def restore(self):
        with torch.no_grad():
            for t, s in zip(self.tensors, self.saved):
                t.copy_(s)
            for o, saved in zip(self.optimizers, self.state):
                for p, st in o.state.items():
                    old = saved.get(id(p))
                    for k, v in st.items():
                        if not torch.is_tensor(v):
                            if old is not None:
                                st[k] = old[k]
                            continue
                        if old is not None and torch.is_tensor(old.get(k)):
                            v.copy_(old[k])
                        else:
                            v.zero_()


_GRAPH_GROUPS = {}


def graph_group(group, device):
    """A process group over the same ranks as ``group`` reserved for collectives captured in HIP
    graphs (created once per (group, device), on every rank at the same point: the first capture,
    outside the capture itself).  The group is always created with ``device_id``: with the default
    group bound to a device (``init_process_group(..., device_id=dev)``) its RCCL communicator is
    split off eagerly, and without that binding torch connects the new communicator eagerly
    (``eager_connect_single_device``) -- either way no communicator is created inside a capture,
    and no eager collective ever runs on this group.  gloo groups are returned unchanged (gloo
    collectives cannot be captured)."""
    if dist.get_backend(group) != "nccl":
        return group
    device = torch.device(device)
    if device.index is None:
        device = torch.device(device.type, torch.cuda.current_device())
    key = (id(group), str(device))
    if key not in _GRAPH_GROUPS:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("graph_group: create the graph collectives' group before the capture begins")
        ranks = None if group is None else dist.get_process_group_ranks(group)
        _GRAPH_GROUPS[key] = dist.new_group(ranks=ranks, backend="nccl", device_id=device,
                                            group_desc="vo_graph_collectives")
    return _GRAPH_GROUPS[key]


def _warmup_ctx(bucketers):
    stack = contextlib.ExitStack()
    for b in bucketers:
        if b is not None:
            stack.enter_context(b.warmup())
    return stack


def _capture_ctx(bucketers):
    stack = contextlib.ExitStack()
    for b in bucketers:
        if b is not None:
            stack.enter_context(b.capturing())
    return stack


def _check_graph_runtime():
    import visual_onoma_to_wave_amd as _pkg
    if _pkg.PACKET_CAPTURE_SET_LATE:
        raise RuntimeError(
            "HIP-graph training: visual_onoma_to_wave_amd was imported after torch had initialised the HIP "
            "runtime, so its DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 setting came too late to take effect. Import the "
            "package (or export DEBUG_CLR_GRAPH_PACKET_CAPTURE=0) before the first CUDA call, e.g. before "
            "torch.cuda.set_device(local_rank); with the CLR packet-capture launch path replays of the training "
            "step compute wrong values (DESIGN.md section 7)")
    if not packet_capture_disabled():
        raise RuntimeError(
            "HIP-graph training needs DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 in effect when the HIP runtime "
            "initialises (visual_onoma_to_wave_amd sets it on import: import the package, or export the "
            "variable, before the first CUDA call); with the CLR packet-capture launch path replays of the "
            "training step compute wrong values (DESIGN.md section 7)")


class GraphedTrainStep:
    """``train_step`` replayed as one HIP graph: forward, loss, backward (with ``bucketer``'s RCCL
    all-reduces under torchrun), clip and the Adam update are captured once after ``warmup``
    eager steps on a side stream whose effects are then undone (``TrainState``); each call copies
    the batch into the graph's static tensors, advances the learning-rate schedule (a device
    tensor, ``ScheduledOptim(capturable=True)``) and replays -- exactly one update per call, no
    host synchronisation.  The acoustic step launches ~1.9k kernels, so the eager loop is bound
    by host launch time.  Returns the graph's loss tensors (overwritten by the next call)."""

    def __init__(self, model, optimizer, loss_fn, grad_clip=1.0, use_image=True, warmup=3, bucketer=None):
        _check_graph_runtime()
        self.model, self.opt, self.loss_fn = model, optimizer, loss_fn
        self.grad_clip, self.use_image, self.warmup = grad_clip, use_image, warmup
        self.bucketer = bucketer
        self.graph = None

    def _body(self, batch):
        output = self.model(*(batch[1:]), self.use_image)
        losses = self.loss_fn(batch, output)
        losses[0].backward()
        if self.bucketer is not None:
            self.bucketer.finish()
        params = [p for p in self.model.parameters() if p.grad is not None]
        torch.nn.utils.clip_grad_norm_(params, self.grad_clip)
        self.opt._optimizer.step()
        self.opt._optimizer.zero_grad(set_to_none=True)
        return losses

    def _capture(self, batch):
        self.static = tuple(b.clone() if torch.is_tensor(b) else b for b in batch)
        snap = TrainState([self.model], [self.opt._optimizer])
        step0 = self.opt.current_step
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), _warmup_ctx([self.bucketer]):
            for _ in range(self.warmup):
                self.opt._update_learning_rate()
                self._body(self.static)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        AG.reset_packs()  # the capture packs the weights inside the graph (autograd's step-batched packs)
        with _capture_ctx([self.bucketer]), torch.cuda.graph(self.graph):
            self.out = self._body(self.static)
        AG.reset_packs()
        snap.restore()  # the warm-up updates are undone: the first replay is the first update
        self.opt.current_step = step0
        _base.invalidate_packs(self.model)

    def __call__(self, batch):
        if self.graph is None:
            self._capture(batch)
        for s, b in zip(self.static, batch):
            if torch.is_tensor(s):
                s.copy_(b)
            elif s != b:
                raise ValueError("GraphedTrainStep: non-tensor batch entries are fixed at capture")
        self.opt._update_learning_rate()
        self.graph.replay()
        _base.invalidate_packs(self.model)  # replays move the parameters without bumping their versions
        AG.reset_packs()
        return self.out


def init_distributed():
    """torchrun environment -> (rank, world, local_rank); RCCL on GPUs, gloo on CPU."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if torch.cuda.is_available():
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    return rank, world, local
