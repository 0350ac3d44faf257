import os, sys, collections
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests"); sys.path.insert(0, "/root/repo/tests/golden")
import torch
import bench
from visual_onoma_to_wave_amd._base import HipModule
calls = collections.Counter()
orig = HipModule._packed
def patched(self, device, builder, dtype=None):
    cache = self.__dict__.get("_pack_cache", {})
    key = (str(device), dtype or self.compute_dtype, self._params_version())
    if cache.get("key") != key:
        calls[(type(self).__name__, str(dtype or self.compute_dtype), "miss" if cache else "first")] += 1
    return orig(self, device, builder, dtype)
HipModule._packed = patched
dev = torch.device("cuda")
m, g = bench.build_models(dev, "mixed")
args = bench.make_batch(1, 4, 12, 64, dev)
with torch.no_grad():
    for i in range(3):
        calls.clear()
        bench.step(m, g, args)
        torch.cuda.synchronize()
        print(i, dict(calls))
