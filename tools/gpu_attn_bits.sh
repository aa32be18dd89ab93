# attention backward ReLU masks from LDS bits: parity, timing A/B vs tools/ab/libsavqa_base.so,
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the fp32 cfg-2 backward, both libraries
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
B=tools/ab/libsavqa_base.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_model_gpu.py tests/test_precision_gpu.py -k "attn or gattn or block or model or precision or golden" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
for L in new base; do
  if [ $L = base ]; then export SAVQA_LIB=$B; else unset SAVQA_LIB; fi
  echo "== $L"
  timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
  timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
  A="tools/attn_bench.py --T 73"
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/attn_${L}_f -o f -- python3 $A > /dev/null 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/attn_${L}_w -o w -- python3 $A > /dev/null 2>&1
done
unset SAVQA_LIB
python tools/pmc_table.py gpurun_out/pmc/attn_new_f gpurun_out/pmc/attn_new_w --match gattn_bwd | tee gpurun_out/attn_traffic_new.txt
python tools/pmc_table.py gpurun_out/pmc/attn_base_f gpurun_out/pmc/attn_base_w --match gattn_bwd | tee gpurun_out/attn_traffic_base.txt
