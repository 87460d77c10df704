"""Drive tools/probe_fill.hip: LDS-fill rate of the row-GEMM DMA pattern (diagnostic)."""
import ctypes as C
import subprocess
import sys

import torch

SO = "tools/libprobe_fill.so"
if len(sys.argv) > 1 and sys.argv[1] == "build":
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    "-o", SO, "tools/probe_fill.hip"], check=True)
    sys.exit(0)
L = C.CDLL(SO)
M = 32768
sink = torch.zeros(512, dtype=torch.int32, device="cuda")
for N, K, zero in [(1536, 512, 0), (512, 2048, 0), (1536, 512, 1)]:
    A = torch.randint(-127, 128, (M, K), dtype=torch.int8, device="cuda")
    W = torch.randint(-127, 128, (N, K), dtype=torch.int8, device="cuda")
    if zero:
        A.zero_()
        W.zero_()
        print("zero operands:")
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for mode, name in [(1, "dma"), (5, "dma nowait"), (9, "dma Wtiled"), (13, "dma Wtiled nowait"),
                       (2, "mfma only"), (3, "dma+mfma"), (11, "dma+mfma Wtiled"),
                       (18, "mfma only upfront"), (19, "dma+mfma upfront"), (34, "mfma regs only")]:
        f = lambda: L.probe_fill(mode, C.c_void_p(A.data_ptr()), C.c_void_p(W.data_ptr()), M, N, K,
                                 C.c_void_p(sink.data_ptr()), st)
        for _ in range(3):
            assert f() == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            f()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 20 / 1e3
        nblk = (N // 512) * (M // 128)
        byts = nblk * (128 + 512) * K
        print(f"N={N} K={K} {name:18s} {t * 1e6:7.1f} us  fill {byts / t / 1e12:6.2f} TB/s "
              f"({byts / t / 256 / 2.1e9:5.1f} B/clk/CU @2.1GHz)  mfma {2 * M * N * K / t / 5.03e15 * 100:5.1f}%")
