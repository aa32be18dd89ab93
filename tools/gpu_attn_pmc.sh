# attention kernels in isolation: timings (fp32 cfg-2, bf16 cfg-3 shapes) + PMC passes over
# the bf16 backward (usage: bash tools/gpu_attn_pmc.sh TAG)
set -e
T=${1:-attn}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
timeout -k 10 120 python -u tools/attn_bench.py
timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512
A="tools/attn_bench.py --bf16 --B 512 --T 73"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/${T}_kt -o kt -- python3 $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/pmc/${T}_sq -o sq -- python3 $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc/${T}_g -o g -- python3 $A > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc/${T}_m -o m -- python3 $A > /dev/null 2>&1
echo done $T
