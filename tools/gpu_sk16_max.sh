# in-step skinny GEMM times for several 16x16-tile thresholds (SAVQA_SK16_MAX)
set -e
mkdir -p gpurun_out
for mx in 192 257 1100; do
  SAVQA_SK16_MAX=$mx timeout -k 10 200 python -u tools/gemm_breakdown.py > gpurun_out/gb_$mx.txt 2>&1
  echo "== $mx $(grep total gpurun_out/gb_$mx.txt)"
  grep skinny gpurun_out/gb_$mx.txt | head -12
done
