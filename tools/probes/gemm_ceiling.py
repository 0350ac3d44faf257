"""Practical MFMA ceiling on this box: hipBLASLt bf16 GEMMs shaped like the MRF convs as
im2col GEMMs (M = frames, K = taps x C_in, N = C_out)."""
import torch

def t(M, K, N, n=20):
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(K, N, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        a @ b
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(n):
        a @ b
    e.record(); torch.cuda.synchronize()
    ms = s.elapsed_time(e) / n
    print(f"M={M} K={K} N={N}: {ms:.3f} ms  {2*M*K*N/ms/1e9:.1f} TF/s", flush=True)

for (M, K, N) in [(1048576, 128 * 11, 128), (1048576, 128 * 3, 128), (2097152, 64 * 11, 64),
                  (524288, 256 * 11, 256), (524288, 256 * 3, 256), (8192, 8192, 8192), (65536, 4096, 4096)]:
    t(M, K, N)
