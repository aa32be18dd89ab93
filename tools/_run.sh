set -eo pipefail
for s in 0 3 7 9 1 2; do
WPERTURB=1 NO_CPU32=1 SEED=$s timeout -k 10 600 python -u tools/cfg2_fp64_check.py > gpurun_out/fp64w_s$s.txt 2>&1 || { tail -30 gpurun_out/fp64w_s$s.txt; exit 1; }
echo "== seed $s"; grep -v "amdgpu.ids\|oracle torch\|logits max" gpurun_out/fp64w_s$s.txt
done
