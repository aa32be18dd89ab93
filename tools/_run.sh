set -eo pipefail
for r in 1 2; do
for v in base lpold; do
L=structured-alignment-vqa_amd/libsavqa.so; [ $v = lpold ] && L=tools/ab/libsavqa_lpold.so
SAVQA_LIB=$L timeout -k 10 300 python -u tools/gemm_breakdown.py cfg3 > gpurun_out/bd_$v.txt 2>&1 || { tail -20 gpurun_out/bd_$v.txt; exit 1; }
echo "== $v"; grep -E "total|92160x304x1024" gpurun_out/bd_$v.txt
done; done
for r in 1 2; do
for v in base lpold; do
L=structured-alignment-vqa_amd/libsavqa.so; [ $v = lpold ] && L=tools/ab/libsavqa_lpold.so
SAVQA_LIB=$L timeout -k 10 300 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$v cfg3', d['value'])"
done; done
