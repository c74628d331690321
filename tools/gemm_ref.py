"""Reference points for the MFMA roofline: torch (hipBLASLt) bf16 GEMMs, square and the conv's own
implicit-GEMM shapes (M = N*T*V rows, N = Cout, K = Kt*Cin)."""
import torch
dev = "cuda:0"
for (M, N, K) in [(8192, 8192, 8192), (240000, 128, 1152), (120000, 256, 2304), (480000, 64, 576)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 20
    s.record()
    for _ in range(reps):
        c = a @ b
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    print(f"GEMM {M}x{N}x{K}: {ms*1e3:8.1f} us  {2*M*N*K/ms/1e9:8.1f} TFLOP/s", flush=True)
