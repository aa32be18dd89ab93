# Kernel trace + three SQ PMC passes (each its own run) over one command.
# usage: bash tools/pmc_passes.sh TAG CMD...   (outputs under gpurun_out/pmc/TAG_*)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
T=$1; shift
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/${T}_kt -o kt -- "$@" > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/${T}_sq -o sq -- "$@" > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/pmc/${T}_g -o g -- "$@" > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pmc/${T}_w -o w -- "$@" > /dev/null 2>&1 || echo "pass 4 failed"
echo done $T
