"""Library reference point: torch._int_mm (hipBLASLt int8 -> int32, no epilogue) on the
cfg3 QuantLinear shapes, us and % of the nominal int8 MFMA peak."""
import torch

PEAK = 256 * 4096 * 2 * 2.4e9
M = 256 * 128
for name, N, K in [("QKV", 1536, 512), ("O", 512, 512), ("FFN1", 2048, 512), ("FFN2", 512, 2048)]:
    a = torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda")
    b = torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda").t()
    try:
        for _ in range(3):
            torch._int_mm(a, b)
    except Exception as e:  # noqa: BLE001
        print(f"{name}: _int_mm unavailable ({type(e).__name__}: {e})")
        continue
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        torch._int_mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / 10
    print(f"_int_mm {name:5s} {t * 1e6:7.1f} us  {100 * 2 * M * N * K / t / PEAK:5.1f} % of int8 peak")
