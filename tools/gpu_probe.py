import torch, time, sys
torch.ops.load_library('solvingpapers_amd/_C.so')
print(torch.cuda.get_device_name(0), torch.cuda.get_device_properties(0).gcnArchName, flush=True)
for D in (256, 768, 4096):
    x = torch.randn(1000, D, device='cuda', dtype=torch.bfloat16)
    r = torch.randn(1000, D, device='cuda', dtype=torch.bfloat16)
    w = torch.randn(D, device='cuda', dtype=torch.bfloat16)
    y, h, rstd, mean = torch.ops.spa.norm_fwd(x, r, w, None, 1e-5)
    hr = (x.float() + r.float()).bfloat16().float()
    ref = hr * torch.rsqrt(hr.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    print(D, (y.float() - ref).abs().max().item(), (h.float()-hr).abs().max().item(), flush=True)
x = torch.randn(8192, 4096, device='cuda', dtype=torch.bfloat16)
w = torch.randn(4096, device='cuda', dtype=torch.bfloat16)
for _ in range(3): torch.ops.spa.norm_fwd(x, None, w, None, 1e-5)
torch.cuda.synchronize(); t=time.time()
for _ in range(50): torch.ops.spa.norm_fwd(x, None, w, None, 1e-5)
torch.cuda.synchronize(); dt=(time.time()-t)/50
print('norm fwd 8192x4096 us', dt*1e6, 'GB/s', 2*x.numel()*2/dt/1e9)
a = torch.randn(8192, 4096, device='cuda', dtype=torch.bfloat16); b = torch.randn(4096, 14336, device='cuda', dtype=torch.bfloat16)
for _ in range(3): a@b
torch.cuda.synchronize(); t=time.time()
for _ in range(20): a@b
torch.cuda.synchronize(); dt=(time.time()-t)/20
print('gemm 8192x4096x14336 TF', 2*8192*4096*14336/dt/1e12)
