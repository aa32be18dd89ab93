# attention ReLU bits (124 VGPRs) + fp32 small-tile tail + lp PRE without tail code:
# parity, attention timings / traffic, step A/B (new vs nosmall vs base)
set -eo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
B=tools/ab/libsavqa_base.so
NS=tools/ab/libsavqa_nosmall.so
timeout -k 10 400 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_blocks_gpu.py tests/test_model_gpu.py tests/test_precision_gpu.py tests/test_gemm_lp_gpu.py -k "attn or gattn or block or model or precision or golden or gemm or lp or bf16 or fp8" > gpurun_out/ab3_tests.log 2>&1 || { tail -30 gpurun_out/ab3_tests.log; exit 1; }
tail -2 gpurun_out/ab3_tests.log
echo "== attn new"; timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
echo "== attn base"; SAVQA_LIB=$B timeout -k 10 120 python -u tools/attn_bench.py 2>&1 | grep -v amdgpu.ids
SAVQA_LIB=$B timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
A="tools/attn_bench.py --T 73"
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/attn2_new_f -o f -- python3 $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/attn2_new_w -o w -- python3 $A > /dev/null 2>&1
python tools/pmc_table.py gpurun_out/pmc/attn2_new_f gpurun_out/pmc/attn2_new_w --match gattn_bwd | tee gpurun_out/attn2_traffic_new.txt
for r in 1 2; do
  for L in new nosmall base; do
    if [ $L = base ]; then export SAVQA_LIB=$B; elif [ $L = nosmall ]; then export SAVQA_LIB=$NS; else unset SAVQA_LIB; fi
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L cfg2', d['value'])"
  done
  unset SAVQA_LIB
  timeout -k 10 200 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new cfg3', d['value'])"
  SAVQA_LIB=$B timeout -k 10 200 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base cfg3', d['value'])"
done
timeout -k 10 200 python -u tools/lp_bench.py 2>&1 | grep -v amdgpu.ids | grep -E "resid|total"
