set -eo pipefail
export SAVQA_BENCH_PREC=fp32x6
S="NT:18688:2048:512 NN:18688:512:2048 TN:2048:512:18688 NT:18688:1536:512"
for r in 1 2; do for L in structured-alignment-vqa_amd/libsavqa.so tools/ab/libsavqa_p1.so tools/ab/libsavqa_p2.so; do
echo "== $L"; SAVQA_LIB=$L timeout -k 10 200 python -u tools/gemm_bench.py $S 2>&1 | grep -v amdgpu.ids | cut -c1-70
done; done
for r in 1 2; do for L in structured-alignment-vqa_amd/libsavqa.so tools/ab/libsavqa_p1.so tools/ab/libsavqa_p2.so; do
SAVQA_LIB=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$L cfg2', d['value'])"
done; done
