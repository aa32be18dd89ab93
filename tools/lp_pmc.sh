# PMC passes over one savqa_gemm_lp shape (usage: bash tools/lp_pmc.sh LAYOUT M N K OUT HINT TAG)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
A="$1 $2 $3 $4 $5 $6"; T=$7
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/${T}_kt -o kt -- python3 tools/lp_one.py $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/${T}_sq -o sq -- python3 tools/lp_one.py $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmc/${T}_g -o g -- python3 tools/lp_one.py $A > /dev/null 2>&1
echo done $T
