import torch, time
dev='cuda'
def bench(M,N,K,iters=50):
    a=torch.randn(M,K,device=dev,dtype=torch.bfloat16); b=torch.randn(N,K,device=dev,dtype=torch.bfloat16)
    for _ in range(5): c=a@b.t()
    torch.cuda.synchronize(); s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): c=a@b.t()
    e.record(); torch.cuda.synchronize(); ms=s.elapsed_time(e)/iters
    print(f"M={M} N={N} K={K}: {ms*1e3:.1f} us  {2*M*N*K/ms/1e9:.1f} TF/s", flush=True)
for (M,N,K) in [(21984,3072,1024),(21984,1024,1024),(21984,4096,1024),(21984,1024,4096),(8192,8192,8192),(16384,16384,4096)]:
    bench(M,N,K)
