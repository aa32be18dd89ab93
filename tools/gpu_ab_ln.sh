set -eo pipefail
for V in base ln1024_32 ln2048_32 ln2048_64; do
  L=structured-alignment-vqa_amd/libsavqa.so; [ $V != base ] && L=tools/ab/libsavqa_$V.so
  echo "== $V"; SAVQA_LIB=$L timeout -k 10 120 python -u tools/ln_bench.py 2>&1 | grep -v amdgpu.ids | grep -i bwd
done
for r in 1 2; do for V in base ln2048_32; do
  L=structured-alignment-vqa_amd/libsavqa.so; [ $V != base ] && L=tools/ab/libsavqa_$V.so
  SAVQA_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$V bench', d['value'])"
done; done
