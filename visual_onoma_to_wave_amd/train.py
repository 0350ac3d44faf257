"""Data-parallel training step (config C4; reference: scripts/04_train.py:115-175).

The reference trains with single-process ``nn.DataParallel`` (GPU0 broadcasts 141 MB of
parameters and reduce-adds 139 MB of gradients every step, 04_train.py:75).  Here: one
process per GPU (torchrun), parameters broadcast once, and a bucketed gradient all-reduce
over RCCL/xGMI launched from per-parameter post-accumulate hooks, so each bucket's
collective overlaps the rest of the backward on a separate stream.  Buckets are ~25 MB
(about 6 for the 139 MB of fp32 gradients): large enough to run near link bandwidth on the
7 point-to-point xGMI links, small enough that the first bucket starts early.  Parameters
that receive no gradient on the path (``encoder.src_word_emb`` with image input,
``variance_adaptor.kurt_embedding`` without kurtosis conditioning) are left out.
"""

import torch
import torch.distributed as dist


class GradBucketer:
    """Bucketed, backward-overlapped gradient averaging across the default process group."""

    def __init__(self, params, bucket_mb=25.0, group=None):
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
        self.flat = [None] * len(self.buckets)
        self.pending = [0] * len(self.buckets)
        self.works = []
        self.side = torch.cuda.Stream() if self.params and self.params[0].is_cuda else None
        self.hooks = [p.register_post_accumulate_grad_hook(self._ready) for p in self.params]
        self.reset()

    def reset(self):
        self.pending = [len(b) for b in self.buckets]
        self.works = []

    def broadcast_parameters(self, module):
        for t in list(module.parameters()) + list(module.buffers()):
            dist.broadcast(t.data, 0, group=self.group)

    def _launch(self, i):
        b = self.buckets[i]
        main = torch.cuda.current_stream() if self.side is not None else None
        if self.side is not None:
            self.side.wait_stream(main)
            ctx = torch.cuda.stream(self.side)
        else:
            ctx = _Null()
        with ctx:
            flat = torch.cat([p.grad.reshape(-1).float() for p in b])
            flat.div_(self.world)
            work = dist.all_reduce(flat, group=self.group, async_op=True)
        self.flat[i] = flat
        self.works.append((i, work))

    def _ready(self, p):
        i = self.bucket_of[id(p)]
        self.pending[i] -= 1
        if self.pending[i] == 0:
            self._launch(i)

    def finish(self):
        """Wait for every bucket, scatter the averaged gradients back (call after backward)."""
        for i, n in enumerate(self.pending):
            if n > 0:  # parameters that got no gradient this step
                for p in self.buckets[i]:
                    if p.grad is None:
                        p.grad = torch.zeros_like(p)
                self._launch(i)
        for i, work in self.works:
            work.wait()
            off = 0
            for p in self.buckets[i]:
                n = p.numel()
                p.grad.copy_(self.flat[i][off: off + n].view_as(p.grad))
                off += n
        if self.side is not None:
            torch.cuda.current_stream().wait_stream(self.side)
        self.reset()


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


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


def graph_fence():
    """Host wait for a HIP-graph replay to finish, called right after ``replay()``.  Measured
    on this ROCm: back-to-back replays of the acoustic step without it produced NaN losses after
    ~10 steps; an event recorded after the replay and waited on before the next one did not
    prevent it, a stream synchronize does (graphed and eager steps then match).  Costs ~1 %."""
    torch.cuda.current_stream().synchronize()
    return None


class GraphedTrainStep:
    """``train_step`` replayed as one HIP graph (single process): forward, loss, backward, clip
    and the Adam update are captured once after ``warmup`` eager steps on a side stream; each
    call copies the batch into the graph's static tensors, advances the learning-rate schedule
    (a device tensor, ``ScheduledOptim(capturable=True)``) and replays.  The acoustic step
    launches ~1.9k kernels, so the eager loop is bound by host launch time.  Returns the
    graph's loss tensors (overwritten by the next call)."""

    def __init__(self, model, optimizer, loss_fn, grad_clip=1.0, use_image=True, warmup=3):
        self.model, self.opt, self.loss_fn = model, optimizer, loss_fn
        self.grad_clip, self.use_image, self.warmup = grad_clip, use_image, warmup
        self.graph = None

    def _body(self, batch):
        output = self.model(*(batch[1:]), self.use_image)
        losses = self.loss_fn(batch, output)
        losses[0].backward()
        params = [p for p in self.model.parameters() if p.grad is not None]
        torch.nn.utils.clip_grad_norm_(params, self.grad_clip)
        self.opt._optimizer.step()
        self.opt._optimizer.zero_grad(set_to_none=True)
        return losses

    def __call__(self, batch):
        if self.graph is None:
            self.static = tuple(b.clone() if torch.is_tensor(b) else b for b in batch)
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(self.warmup):
                    self.opt._update_learning_rate()
                    self._body(self.static)
            torch.cuda.current_stream().wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self.out = self._body(self.static)
        if getattr(self, "done", None) is not None:
            self.done.synchronize()  # see graph_fence
        for s, b in zip(self.static, batch):
            if torch.is_tensor(s):
                s.copy_(b)
            elif s != b:
                raise ValueError("GraphedTrainStep: non-tensor batch entries are fixed at capture")
        self.opt._update_learning_rate()
        self.graph.replay()
        self.done = graph_fence()
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
