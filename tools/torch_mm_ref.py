import torch, time
dev='cuda'
for (M,N,K) in [(43840,1536,384),(43840,1152,384),(43840,384,1536),(43840,384,384),(8192,8192,8192),(4096,4096,4096)]:
    a=torch.randn(M,K,device=dev,dtype=torch.float16); w=torch.randn(N,K,device=dev,dtype=torch.float16)
    for _ in range(5): y=torch.nn.functional.linear(a,w)
    torch.cuda.synchronize()
    e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): y=torch.nn.functional.linear(a,w)
    e1.record(); torch.cuda.synchronize()
    ms=e0.elapsed_time(e1)/20
    print(f"torch linear M{M} N{N} K{K}: {ms*1e3:.1f} us {2*M*N*K/ms/1e9:.1f} TF/s", flush=True)
