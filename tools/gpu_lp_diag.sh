# Where the 128x128 lp kernel's time goes: diagnostic builds (no MFMA / no k-loop DMA / no
# epilogue) on cfg-3 shapes, plus SQ PMC passes of the K=512 bf16-out forward and the dW
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/lp_bench.py --dbg1 > gpurun_out/lp_dbg1.log 2>&1 || { tail -20 gpurun_out/lp_dbg1.log; exit 1; }
grep -v amdgpu gpurun_out/lp_dbg1.log
bash tools/lp_pmc.sh NT 37376 2048 512 bf16 1 ffn1
bash tools/lp_pmc.sh TN 2048 512 37376 atomic 0 dwffn1
python tools/pmc_table.py gpurun_out/pmc 2>/dev/null | tee gpurun_out/lp_pmc_table.txt || true
