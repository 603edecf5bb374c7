"""fp32 GEMM rates of torch.mm (rocBLAS / hipBLASLt) at the PPO-update shapes (tokens = 4096 x 5)."""
import os
import time
import torch

dev = torch.device("cuda")
T = 20480
shapes = [  # (M, K, N, label)
    (T, 128, 384, "qkv fwd"), (T, 384, 128, "qkv dX"), (384, T, 128, "qkv dW (K=tok)"),
    (T, 128, 128, "out fwd"), (128, T, 128, "out dW"),
    (T, 128, 256, "ffn1 fwd"), (T, 256, 128, "ffn2 fwd"), (256, T, 128, "ffn1 dW"), (128, T, 256, "ffn2 dW"),
    (4096, 128, 256, "pruned ffn1"), (4096, 128, 128, "pruned out"),
]
for backend in os.environ.get("BACKENDS", "default,cublaslt,cublas").split(","):
    if backend != "default":
        try:
            torch.backends.cuda.preferred_blas_library(backend)
        except Exception as e:
            print("backend", backend, "unavailable", e)
            continue
    print("== backend", torch.backends.cuda.preferred_blas_library())
    for M, K, N, lab in shapes:
        if "dW" in lab:
            a = torch.randn(K, M, device=dev).t()  # dY^T view: [M][K] with K-major storage
        else:
            a = torch.randn(M, K, device=dev)
        b = torch.randn(K, N, device=dev)
        for _ in range(3):
            c = a @ b
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            c = a @ b
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(f"{lab:16s} M={M:6d} K={K:6d} N={N:4d}: {dt * 1e6:8.1f} us  {2 * M * K * N / dt / 1e12:6.1f} TF/s", flush=True)
