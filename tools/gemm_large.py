import torch, time
def t(f, reps=10):
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0,e1=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1)/reps*1e-3
M,K,N=245760,512,512
x=torch.randn(M,K,device='cuda'); W=torch.randn(N,K,device='cuda'); b=torch.randn(N,device='cuda')
gy=torch.randn(M,N,device='cuda')
fl=2*M*N*K
for name,f in [("fwd addmm x@W^T",lambda: torch.addmm(b,x,W.t())),
               ("fwd mm x@W^T",lambda: torch.mm(x,W.t())),
               ("fwd swapped (W@x^T)^T",lambda: torch.mm(W,x.t()).t()),
               ("dgrad gy@W",lambda: torch.mm(gy,W)),
               ("dgrad swapped (W^T gy^T)^T",lambda: torch.mm(W.t(),gy.t()).t()),
               ("wgrad gy^T x",lambda: torch.mm(gy.t(),x)),
               ("wgrad bmm16",lambda: torch.bmm(gy.view(16,-1,N).transpose(1,2),x.view(16,-1,K)).sum(0)),
               ("wgrad bmm32",lambda: torch.bmm(gy.view(32,-1,N).transpose(1,2),x.view(32,-1,K)).sum(0)),
               ("wgrad bmm64",lambda: torch.bmm(gy.view(64,-1,N).transpose(1,2),x.view(64,-1,K)).sum(0)),
               ("fwd N=256",lambda: torch.mm(x,W[:256].t())),
               ("fwd K=768",lambda: torch.mm(torch.randn(1,1,device='cuda').expand(1,1) if False else x2,W2.t())),
               ]:
    if name=="fwd K=768":
        continue
    s=t(f); ff=fl/2 if "N=256" in name else fl
    print(f"{name:32s} {s*1e6:8.1f} us {ff/s/1e12:6.1f} TF/s",flush=True)
