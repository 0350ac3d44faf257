"""Adam / AdamW whose update runs as multi-tensor HIP launches (``vo_adam_multi``).

Replaces ``torch.optim.Adam`` behind ``ScheduledOptim`` (scripts/model/optimizer.py:9-15; config C4)
and the HiFi-GAN V1 recipe's ``torch.optim.AdamW`` (config C5): one launch per 64 tensors instead
of PyTorch's per-op multi-tensor kernels, the learning rate and step count read from device
memory (graph-capturable, no host synchronisation).  The state layout is torch's --
``state[p] = {"step", "exp_avg", "exp_avg_sq"}`` and the Adam param-group keys -- so
``state_dict()`` / ``load_state_dict()`` exchange checkpoints with the reference's Adam
(``{"model", "optimizer"}`` files, scripts/04_train.py:160-168).

Semantics: torch's single-tensor Adam / AdamW (amsgrad and maximize off).  One step counter per
param group (every ``state[p]["step"]`` is that group's tensor): parameters are updated together,
as in the training steps here -- ``load_state_dict`` refuses a group whose per-parameter steps
differ, and ``step`` warns when a parameter first gets a gradient after the group's first step.
``load_state_dict`` copies the loaded values into the device tensors a captured step uses -- a capturable
group's learning rate, the group's step tensor and the moments -- so a graph captured before the load
continues from the loaded state; capturing a step with a float learning rate raises.  fp32 parameters,
gradients and moments on the GPU.
"""

import ctypes
import warnings

import torch
from torch.autograd.graph import increment_version

from . import _lib

_P = ctypes.c_void_p


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False,
                 capturable=False):
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False, maximize=False,
                        foreach=None, capturable=capturable, differentiable=False, fused=True,
                        decoupled_weight_decay=bool(decoupled))
        super().__init__(params, defaults)
        self._tables = {}

    # ---- per-group device scalars
    def _group_step(self, group):
        t = group.get("_vo_step")
        if t is None:
            dev = group["params"][0].device
            old = [self.state[p]["step"] for p in group["params"] if "step" in self.state.get(p, {})]
            v = max((float(s) for s in old), default=0.0)
            t = torch.full((), v, dtype=torch.float32, device=dev)
            group["_vo_step"] = t
            for p in group["params"]:
                if "step" in self.state.get(p, {}):
                    self.state[p]["step"] = t
        return t

    def _group_lr(self, group):
        lr = group["lr"]
        if torch.is_tensor(lr):
            return lr if lr.dtype == torch.float32 else lr.float()
        if torch.cuda.is_current_stream_capturing():
            # a float lr would be baked into the graph as a constant: schedule changes between replays
            # would be silently ignored
            raise RuntimeError("FusedAdam: capturing a step needs device-tensor learning rates "
                               "(construct with capturable=True and lr=torch.tensor(...))")
        t = group.get("_vo_lr")
        if t is None:
            t = group["_vo_lr"] = torch.empty((), dtype=torch.float32, device=group["params"][0].device)
        t.fill_(float(lr))
        return t

    def load_state_dict(self, state_dict):
        # every per-parameter step of a group must agree: one step tensor per group drives the bias
        # correction (a parameter loaded with a smaller step would get the wrong correction)
        for i, g in enumerate(state_dict["param_groups"]):
            steps = {float(state_dict["state"][k]["step"]) for k in g["params"]
                     if k in state_dict["state"] and "step" in state_dict["state"][k]}
            if len(steps) > 1:
                raise ValueError(f"FusedAdam: param group {i} has unequal per-parameter steps {sorted(steps)[:4]}; "
                                 "one step count per group is supported")
        # a captured graph reads and writes the device tensors it was captured with -- a capturable group's
        # learning rate, the group's step tensor and every parameter's moments: keep those tensors and
        # copy the loaded values into them (torch's load_state_dict puts a float / the caller's tensors
        # there), so a step captured before the load continues from the loaded state
        lr_tensors = [g["lr"] if torch.is_tensor(g["lr"]) else None for g in self.param_groups]
        step_tensors = [g.get("_vo_step") for g in self.param_groups]
        moments = {p: {k: self.state[p][k] for k in ("exp_avg", "exp_avg_sq") if k in self.state.get(p, {})}
                   for g in self.param_groups for p in g["params"]}
        super().load_state_dict(state_dict)
        for group, lt in zip(self.param_groups, lr_tensors):
            if lt is not None:
                lt.fill_(float(group["lr"]))
                group["lr"] = lt
        for group, old_step in zip(self.param_groups, step_tensors):
            group.pop("_vo_step", None)
            group.pop("_vo_lr", None)
            for p in group["params"]:
                st = self.state.get(p, {})
                for k in ("exp_avg", "exp_avg_sq"):
                    keep = moments[p].get(k)
                    if k not in st:
                        if keep is not None:
                            # no loaded moments for a parameter a captured step still reads: zero them
                            # (an eager step would start it from zeros) and keep them in the state
                            keep.zero_()
                            st[k] = keep
                            self.state[p] = st
                        continue
                    if keep is not None and keep.shape == st[k].shape:
                        keep.copy_(st[k])
                        st[k] = keep
                    else:  # own copies: torch's load_state_dict keeps the caller's tensors
                        st[k] = st[k].to(device=p.device, dtype=torch.float32, copy=True).contiguous()
            t = self._group_step(group)
            if old_step is not None:
                old_step.copy_(t)
                group["_vo_step"] = old_step
                for p in group["params"]:
                    if "step" in self.state.get(p, {}):
                        self.state[p]["step"] = old_step
        self._tables.clear()

    def state_dict(self):
        sd = super().state_dict()
        for g in sd["param_groups"]:
            for k in ("_vo_step", "_vo_lr", "_vo_started", "_vo_warned"):
                g.pop(k, None)
        return sd

    def _table(self, ps, gs, ms, vs):
        key = tuple(t.data_ptr() for t in ps + gs + ms + vs)
        tab = self._tables.get(key)
        if tab is None:
            n = len(ps)
            arrs = ((_P * n)(*[t.data_ptr() for t in ps]), (_P * n)(*[t.data_ptr() for t in gs]),
                    (_P * n)(*[t.data_ptr() for t in ms]), (_P * n)(*[t.data_ptr() for t in vs]),
                    (ctypes.c_int64 * n)(*[t.numel() for t in ps]))
            tab = (arrs, [ctypes.cast(a, _P) for a in arrs])
            if len(self._tables) > 64:
                self._tables.clear()
            self._tables[key] = tab
        return tab

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            if group.get("amsgrad") or group.get("maximize"):
                raise NotImplementedError("FusedAdam: amsgrad / maximize are not supported")
            ps, gs, ms, vs = [], [], [], []
            step_t = self._group_step(group)
            for p in group["params"]:
                if p.grad is None:
                    continue
                if not (p.is_cuda and p.dtype == torch.float32 and p.is_contiguous()):
                    raise TypeError("FusedAdam: contiguous fp32 CUDA parameters only")
                g = p.grad
                if g.dtype != torch.float32 or not g.is_contiguous():
                    raise TypeError("FusedAdam: contiguous fp32 gradients only")
                st = self.state[p]
                if "exp_avg" not in st:
                    if group.get("_vo_started") and not group.get("_vo_warned"):
                        warnings.warn("FusedAdam: a parameter got its first gradient after the group's first step; "
                                      "it shares the group's step count (torch's Adam would count its own steps "
                                      "from 1), so its bias correction differs from torch's", RuntimeWarning)
                        group["_vo_warned"] = True
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st["step"] = step_t
                ps.append(p)
                gs.append(g)
                ms.append(st["exp_avg"])
                vs.append(st["exp_avg_sq"])
            if not ps:
                continue
            group["_vo_started"] = True
            b1, b2 = group["betas"]
            lr_t = self._group_lr(group)
            tp, tg, tm, tv, tn = self._table(ps, gs, ms, vs)[1]
            stream = ctypes.c_void_p(torch.cuda.current_stream(ps[0].device).cuda_stream)
            L = _lib.lib()
            _lib.check(L.vo_adam_multi(len(ps), tp, tg, tm, tv, tn, ctypes.c_void_p(lr_t.data_ptr()),
                                       ctypes.c_void_p(step_t.data_ptr()), float(b1), float(b2), float(group["eps"]),
                                       float(group["weight_decay"]), int(bool(group.get("decoupled_weight_decay"))),
                                       stream), "vo_adam_multi")
            _lib.check(L.vo_opt_step_increment(ctypes.c_void_p(step_t.data_ptr()), stream), "vo_opt_step_increment")
            # the kernel writes the parameters behind autograd's back: bump their version counters as
            # torch's in-place updates do, so caches keyed on them (the packed bf16 weights,
            # _base.PackedModule) see the step
            increment_version(ps)
        return loss


def AdamW(params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, capturable=False):
    """torch.optim.AdamW's defaults (weight decay 0.01, decoupled) on the fused HIP update."""
    return FusedAdam(params, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decoupled=True,
                     capturable=capturable)
