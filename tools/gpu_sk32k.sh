# 4-wave 32x32 skinny for short K: parity tests with it on, in-step breakdown and bench A/B
set -e
mkdir -p gpurun_out
SAVQA_SK32_KSMALL=256 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sk32k_tests.log 2>&1 || { tail -30 gpurun_out/sk32k_tests.log; exit 1; }
tail -1 gpurun_out/sk32k_tests.log
for ks in 0 256; do
  SAVQA_SK32_KSMALL=$ks timeout -k 10 200 python -u tools/gemm_breakdown.py > gpurun_out/gb32_ks$ks.txt 2>&1
  echo "== $ks $(grep total gpurun_out/gb32_ks$ks.txt)"
  grep -E "x256 " gpurun_out/gb32_ks$ks.txt | head -5
done
for ks in 0 256 0 256; do
  SAVQA_SK32_KSMALL=$ks timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench32_ks$ks.json 2> gpurun_out/bench32_ks$ks.err
  echo "ks $ks: $(python -c "import json;d=json.load(open('gpurun_out/bench32_ks$ks.json'));print(d['value'],d['ms_per_step'])")"
done
