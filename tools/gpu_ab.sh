# A/B of a variant libsavqa (tools/ab/libsavqa_*.so) against the in-tree one on the cfg-2
# GEMM shapes and the cfg-2 bench step, interleaved (usage: bash tools/gpu_ab.sh VARIANT)
set -eo pipefail
mkdir -p gpurun_out
V=${1:-prio}
for r in 1 2; do
  echo "== base $r"; timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | tail -14
  echo "== $V $r"; SAVQA_LIB=tools/ab/libsavqa_$V.so timeout -k 10 120 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | tail -14
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base bench', d['value'])"
  SAVQA_LIB=tools/ab/libsavqa_$V.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-roofline | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$V bench', d['value'])"
done
