set -o pipefail
mkdir -p gpurun_out/r05e
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r05e/ffn_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r05e/ffn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ffn_ab.py 3 > gpurun_out/r05e/ffn_ab.log 2>&1; rc=$?; cat gpurun_out/r05e/ffn_ab.log | grep -v amdgpu.ids; exit $rc
