"""Calibration only: hipBLASLt (torch.matmul) TFLOP/s at the config-2 GEMM shapes, for comparison with gemm.hip."""
import torch, time
M=35552
for (N,K) in [(9216,3072),(3072,3072),(12288,3072),(3072,12288)]:
    a=torch.randn(M,K,device='cuda').bfloat16(); w=torch.randn(N,K,device='cuda').bfloat16()*K**-0.5
    for _ in range(3): c=a@w.t()
    torch.cuda.synchronize()
    s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10): c=a@w.t()
    e.record(); torch.cuda.synchronize()
    t=s.elapsed_time(e)/10/1e3
    print(N,K, f"{t*1e3:.3f} ms {2*M*N*K/t/1e12:.0f} TF", flush=True)
