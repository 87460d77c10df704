set -o pipefail
O=gpurun_out/r05g; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ffn.py -x -v --timeout 120 --timeout-method thread > $O/ffn_tests.log 2>&1
rc=$?; grep -E "passed|failed|Error|assert" $O/ffn_tests.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/ffn_ab.py 3 > $O/ffn_ab.log 2>&1; rc=$?; grep -v amdgpu.ids $O/ffn_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/ffn_stamps.py > $O/stamps.log 2>&1; rc=$?; grep -v amdgpu.ids $O/stamps.log; exit $rc
