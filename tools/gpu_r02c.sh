set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/dbg/race_probe.py > gpurun_out/race_conc.log 2>&1; echo "rc=$?"; grep -v amdgpu.ids gpurun_out/race_conc.log | head -8
timeout -k 10 300 python -u -m pytest -x -q -s --timeout 240 --timeout-method thread tests/test_graph_capture_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py 2>&1 | tee gpurun_out/graph_test.log | grep -E "diagnostics|passed|failed|Error"
