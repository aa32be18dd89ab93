# 16x16-tile skinny GEMM: parity tests, standalone A/B (SAVQA_SK16_MAX=0 = 32x32 tiles), bench A/B
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sk16_tests.log 2>&1 || { tail -30 gpurun_out/sk16_tests.log; exit 1; }
tail -2 gpurun_out/sk16_tests.log
S="NN:256:512:2048 NN:256:512:512 TN:512:512:256 NT:256:512:2048 NT:256:2048:512 TN:2048:512:256 NN:256:2048:512 NT:256:512:512 TN:512:2048:256 NN:256:914:512"
for mx in 0 256; do
  echo "== SAVQA_SK16_MAX=$mx"
  SAVQA_SK16_MAX=$mx timeout -k 10 150 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids | awk '{print $1, $6, $7}'
done
for mx in 0 256 0 256; do
  SAVQA_SK16_MAX=$mx timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_sk$mx.json 2> gpurun_out/bench_sk$mx.err
  echo "sk16max $mx: $(python -c "import json;d=json.load(open('gpurun_out/bench_sk$mx.json'));print(d['value'],d['ms_per_step'])")"
done
