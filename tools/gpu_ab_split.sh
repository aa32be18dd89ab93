# A/B: whole-grid slice-major XCD remap of split-K launches (in-tree lib) vs the tile-only
# remap (tools/ab/libsavqa_base.so): lp and fp32 GEMM shapes, then cfg3 / cfg2 bench steps
set -eo pipefail
mkdir -p gpurun_out
B=tools/ab/libsavqa_base.so
timeout -k 10 200 python -u tools/lp_bench.py > gpurun_out/ab_lp_new.log 2>&1
SAVQA_LIB=$B timeout -k 10 200 python -u tools/lp_bench.py > gpurun_out/ab_lp_base.log 2>&1
timeout -k 10 120 python -u tools/gemm_bench.py > gpurun_out/ab_gemm_new.log 2>&1
SAVQA_LIB=$B timeout -k 10 120 python -u tools/gemm_bench.py > gpurun_out/ab_gemm_base.log 2>&1
for r in 1 2; do
  for w in cfg3 cfg2; do
    timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('new $w', d['value'])"
    SAVQA_LIB=$B timeout -k 10 200 python -u bench.py --workload $w --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base $w', d['value'])"
  done
done
