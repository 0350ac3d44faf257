"""Adam with the Noam warm-up / step-anneal schedule (reference: scripts/model/optimizer.py:5-51).

lr(step) = init_lr * min(step^-0.5, warmup^-1.5 * step) * anneal_rate^#{anneal steps < step},
evaluated after the step counter is incremented; Adam(betas, eps, weight_decay) from the
train config.  On the GPU the update runs as multi-tensor HIP launches (``optim.FusedAdam``).
"""

import numpy as np
import torch

from ..optim import FusedAdam


class ScheduledOptim:
    """``capturable=True`` (HIP-graph training, ``train.GraphedTrainStep``): Adam keeps its step
    counts and the learning rate as device tensors, and the schedule writes the new rate into
    that tensor (outside the graph) instead of replacing the Python float."""

    def __init__(self, model, train_config, model_config, current_step, capturable=False):
        o = train_config["optimizer"]
        # every parameter, frozen ones included, as the reference does (scripts/model/optimizer.py:10):
        # the param group then matches a reference checkpoint's optimizer state on resume
        params = list(model.parameters())
        kw = dict(betas=o["betas"], eps=o["eps"], weight_decay=o["weight_decay"])
        if capturable:
            kw.update(capturable=True, lr=torch.tensor(0.0, device=params[0].device))
        if params and params[0].is_cuda:
            # the update as multi-tensor HIP launches (visual_onoma_to_wave_amd.optim), torch Adam's
            # arithmetic and state layout (checkpoints interchange with the reference's Adam)
            self._optimizer = FusedAdam(params, decoupled=False, **kw)
        else:
            self._optimizer = torch.optim.Adam(params, **kw)
        self.n_warmup_steps = o["warm_up_step"]
        self.anneal_steps = o["anneal_steps"]
        self.anneal_rate = o["anneal_rate"]
        self.current_step = current_step
        self.init_lr = o["init_lr"]

    def step_and_update_lr(self):
        self._update_learning_rate()
        self._optimizer.step()

    def zero_grad(self):
        self._optimizer.zero_grad()

    def load_state_dict(self, path):
        self._optimizer.load_state_dict(path)

    def _get_lr_scale(self):
        s = self.current_step
        lr = min(np.power(s, -0.5), np.power(self.n_warmup_steps, -1.5) * s)
        for a in self.anneal_steps:
            if s > a:
                lr = lr * self.anneal_rate
        return lr

    def _update_learning_rate(self):
        self.current_step += 1
        lr = self.init_lr * self._get_lr_scale()
        for group in self._optimizer.param_groups:
            if torch.is_tensor(group["lr"]):
                group["lr"].fill_(lr)
            else:
                group["lr"] = lr
