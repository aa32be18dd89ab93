set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k gemm > gpurun_out/kt.log 2>&1 || { tail -40 gpurun_out/kt.log; exit 1; }
tail -2 gpurun_out/kt.log
bash tools/ab_gemm.sh cur old t14
