set -eo pipefail
SAVQA_BENCH_PREC=fp32x6 timeout -k 10 300 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/x6_shapes.txt
cat gpurun_out/x6_shapes.txt
bash tools/profile_round.sh r05 cfg4
bash tools/profile_round.sh r05 cfg5
bash tools/profile_round.sh r05 rel
