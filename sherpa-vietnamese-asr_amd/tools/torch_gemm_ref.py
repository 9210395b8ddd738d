"""Development probe: time the vendor library (torch.matmul -> hipBLASLt) on the encoder's
projection shapes, bf16 A / bf16 W / bf16 C, to size the headroom of gemm_bf16_kernel."""
import torch
import time

SHAPES = [("ffin1", 98685, 256, 768), ("ffout1", 98685, 768, 256), ("ffin2", 49342, 384, 1536),
          ("ffout2", 49342, 1536, 384), ("ffin3", 24671, 512, 2048), ("ffout3", 24671, 2048, 512),
          ("inproj1", 98685, 256, 272 * 4)]
for name, M, K, N in SHAPES:
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
    af = a.float()
    for label, fn in (("bf16", lambda: a @ w.t()),):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1e3
        by = 2 * (M * K + N * K + M * N)
        print(f"{name:8s} {label} M={M:6d} K={K:5d} N={N:5d} {us:8.1f} us {by / us / 1e3:7.0f} GB/s "
              f"{2 * M * N * K / us / 1e6:7.1f} TF/s", flush=True)
