import sys, torch
sys.path[:0]=['/root/repo','/root/repo/tests']
from visual_onoma_to_wave_amd import autograd as AG, ops
B,T,D,p=4,8,256,0.5
g=torch.Generator(device="cuda").manual_seed(1)
for dual,xdt,rdt in ((True,torch.bfloat16,torch.float32),(False,torch.float32,torch.float32)):
    x=torch.randn(B,T,D,device="cuda",generator=g).to(xdt); res=torch.randn(B,T,D,device="cuda",generator=g).to(rdt)
    gam=torch.ones(D,device="cuda"); bet=torch.zeros(D,device="cuda"); lens=torch.full((B,),T,device="cuda",dtype=torch.int32)
    AG.begin_dropout_step(x.device); seed=AG._DROP["seed"]; salt=AG._DROP["site"]+1
    mask=ops.dropout(torch.ones(B,T,D,device="cuda"),p,seed,salt)!=0
    xc=x.clone().requires_grad_(True); rc=res.clone().requires_grad_(True)
    out=AG.layernorm_drop(xc,rc,gam,bet,lens,p,dual)
    y=out[0] if dual else out
    gy=torch.randn(B,T,D,device="cuda",generator=g)
    dx,=torch.autograd.grad(y,(xc,),gy)
    mm=((dx!=0)!=mask)
    print(dual, "mismatch frac", mm.float().mean().item(), "keep frac", mask.float().mean().item(), "dxnz", (dx!=0).float().mean().item())
    idx=mm.nonzero()[:8].tolist(); print(idx)
    # compare dx!=0 with mask at other salts / shifted index
    for s2 in (salt-1, salt+1, 0):
        m2=ops.dropout(torch.ones(B,T,D,device="cuda"),p,seed,s2)!=0
        print("  salt",s2,"mismatch",((dx!=0)!=m2).float().mean().item())
