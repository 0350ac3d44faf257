import sys, torch
sys.path.insert(0, '.')
from visual_onoma_to_wave_amd import ops
import torch.nn.functional as F
torch.manual_seed(0)
for dt in (torch.float32, torch.bfloat16):
    B, T, Ci, Co, K = 1, 64, 16, 16, 1
    x = torch.randn(B, T, Ci).to(dt).float()
    gy = torch.randn(B, T, Co).to(dt).float()
    ref = torch.nn.grad.conv1d_weight(x.transpose(1, 2), (Co, Ci, K), gy.transpose(1, 2))
    got = ops.conv1d_wgrad(gy.cuda().to(dt), x.cuda().to(dt), K).cpu()
    print(dt, (got - ref).abs().max().item(), ref.abs().max().item())
    if dt == torch.bfloat16:
        # find permutation: compare got[m][n] with ref
        r = ref[:, :, 0]; g = got[:, :, 0]
        print(g[:4, :4]); print(r[:4, :4]); print(r.t()[:4,:4])
