"""Reference point for the encoder GEMMs (methodology: a known-good kernel on the same
hardware): torch._int_mm (hipBLASLt int8 -> int32) at the cfg3 QuantLinear shapes."""
import torch

M = 32768
PEAK = 256 * 4096 * 2 * 2.4e9
for N, K in [(1536, 512), (512, 512), (2048, 512), (512, 2048)]:
    a = torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda")
    b = torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda").t()
    try:
        for _ in range(3):
            c = torch._int_mm(a, b)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            c = torch._int_mm(a, b)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 20 / 1e3
        print(f"_int_mm M={M} N={N} K={K}: {t * 1e6:7.1f} us  {2 * M * N * K / t / PEAK * 100:5.1f}% of int8 peak", flush=True)
    except Exception as ex:
        print(f"_int_mm N={N} K={K}: {type(ex).__name__}: {ex}", flush=True)
