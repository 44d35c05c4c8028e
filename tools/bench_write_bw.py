import torch, time
dev=torch.device("cuda")
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s=time.perf_counter()
    for _ in range(it): fn()
    torch.cuda.synchronize(); return (time.perf_counter()-s)/it
M=802816
x=torch.randn(M,64,device=dev).to(torch.bfloat16)
y=torch.empty(M,256,device=dev,dtype=torch.bfloat16)
z=torch.empty(M,64,device=dev,dtype=torch.bfloat16)
tw=t(lambda: y.fill_(1.0)); print(f"fill 411MB: {tw*1e6:.1f}us {y.numel()*2/tw/1e12:.2f} TB/s")
te=t(lambda: y.view(M,4,64).copy_(x.view(M,1,64).expand(M,4,64))); print(f"expand 103MB->411MB: {te*1e6:.1f}us {(x.numel()+y.numel())*2/te/1e12:.2f} TB/s")
tc=t(lambda: z.copy_(x)); print(f"copy 103MB: {tc*1e6:.1f}us {2*x.numel()*2/tc/1e12:.2f} TB/s")
