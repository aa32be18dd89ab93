# Kernel trace + SQ PMC passes over one savqa_gemm shape
# (usage: bash tools/gemm_pmc.sh LAYOUT M N K PREC TAG)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
A="$1 $2 $3 $4 $5"; T=$6
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/${T}_kt -o kt -- python3 tools/gemm_one.py $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/${T}_sq -o sq -- python3 tools/gemm_one.py $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc/${T}_g -o g -- python3 tools/gemm_one.py $A > /dev/null 2>&1
echo done $T
