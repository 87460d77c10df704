"""Run the decode step's dominant kernel (bench.DOMINANT) 256 times over bench's rotating
operand sets — the program that rocprofv3 PMC passes profile:

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run \
        --output-format csv -- python tools/pmc_dominant.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run \
        --output-format csv -- python tools/pmc_dominant.py
    python tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write > profiles/r03_pmc_dominant.json
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "onnx-transformer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

one, keep = bench.run_dominant(32)
for i in range(256):
    one(i)
torch.cuda.synchronize()
