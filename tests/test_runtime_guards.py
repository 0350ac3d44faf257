"""CPU checks of the host-side runtime guards (round 3):

* the DEBUG_CLR_GRAPH_PACKET_CAPTURE guard: the package records when it set the variable only
  after torch had initialised the HIP runtime (the setting is then dead) and graphed training
  refuses to run in that case;
* ``GradBucketer.warmup()``: warm-up steps before a capture issue no collective;
* ``_base.invalidate_packs(module)``: only the named modules repack after a graph replay."""

import os
import socket
import subprocess
import sys

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_PROBE = r"""
import os, sys, torch
if sys.argv[1] == "late":
    torch.cuda.is_initialized = lambda: True      # as after torch.cuda.set_device() in a user script
import visual_onoma_to_wave_amd as pkg
from visual_onoma_to_wave_amd import train
try:
    train._check_graph_runtime()
    ok = "ok"
except RuntimeError as e:
    ok = "refused:" + ("late" if "too late" in str(e) else "other")
print(pkg.PACKET_CAPTURE_SET_LATE, train.packet_capture_disabled(), ok)
"""


def _probe(mode, preset):
    env = {k: v for k, v in os.environ.items() if k != "DEBUG_CLR_GRAPH_PACKET_CAPTURE"}
    if preset is not None:
        env["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = preset
    r = subprocess.run([sys.executable, "-c", _PROBE, mode], cwd=REPO, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.split()


def test_packet_capture_guard_import_first():
    assert _probe("early", None) == ["False", "True", "ok"]


def test_packet_capture_guard_set_too_late():
    assert _probe("late", None) == ["True", "False", "refused:late"]


def test_packet_capture_guard_user_export_wins():
    # exported by the user before the process started: in effect whatever the import order
    assert _probe("late", "0") == ["False", "True", "ok"]
    assert _probe("early", "1") == ["False", "False", "refused:other"]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _warmup_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from visual_onoma_to_wave_amd.train import GradBucketer, _capture_ctx, _warmup_ctx
    torch.manual_seed(0)
    m = torch.nn.Linear(8, 3)
    bk = GradBucketer(m.parameters(), bucket_mb=0.001)
    calls = []
    real = dist.all_reduce

    def counting(*a, **k):
        calls.append(k.get("group"))
        return real(*a, **k)

    dist.all_reduce = counting
    x = torch.full((2, 8), float(rank + 1))
    with _warmup_ctx([bk, None]):
        m(x).sum().backward()
        bk.finish()
    local = m.weight.grad.clone()
    n_warm = len(calls)
    m.zero_grad(set_to_none=True)
    with _capture_ctx([bk]):               # gloo: the graph group is the bucketer's own group
        m(x).sum().backward()
        bk.finish()
    out[rank] = (n_warm, len(calls), local, m.weight.grad.clone(), bk.local_only, bk.capture_group)
    dist.destroy_process_group()


def test_bucketer_warmup_issues_no_collective():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_warmup_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    for r in range(world):
        n_warm, n_total, local, avg, local_only, cap = out[r]
        assert n_warm == 0 and n_total >= 1 and not local_only and cap is None
        torch.testing.assert_close(local, torch.full_like(local, 2.0 * (r + 1)))   # rank's own grad
        torch.testing.assert_close(avg, torch.full_like(avg, 3.0))                 # mean of 2 and 4


def test_invalidate_packs_per_module():
    from visual_onoma_to_wave_amd import _base

    class M(_base.HipModule):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(2))
            self.builds = 0

        def pack(self):
            def b(device, dtype):
                self.builds += 1
                return self.w.detach().clone()
            return self._packed("cpu", b)

    a, b = M(), M()
    a.pack(), b.pack()
    _base.invalidate_packs(a)
    a.pack(), b.pack()
    assert (a.builds, b.builds) == (2, 1)
    _base.invalidate_packs()
    a.pack(), b.pack()
    assert (a.builds, b.builds) == (3, 2)
