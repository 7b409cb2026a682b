import torch
x=torch.randn(16384,2752,device="cuda").to(torch.bfloat16)
W=torch.randn(1024,2752,device="cuda").to(torch.bfloat16)
b=torch.randn(1024,device="cuda").to(torch.bfloat16)
for _ in range(20): y=torch.addmm(b,x,W.t())
torch.cuda.synchronize()
