# SQ counters of the fp32 GEMM on one cfg-2 shape (own --pmc pass; usage: bash tools/gpu_gemm_pmc.sh)
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/gemm_pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/gemm_pmc -o run -- python3 tools/gemm_bench.py NT:18688:6144:512 TN:6144:512:18688 > gpurun_out/gemm_pmc.log 2>&1
ls gpurun_out/gemm_pmc
