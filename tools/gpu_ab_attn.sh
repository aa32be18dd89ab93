# A/B of attention variant libraries (tools/ab/libsavqa_*.so) against the in-tree one:
# bf16 attention kernels in isolation + the cfg-3 step, interleaved
# (usage: bash tools/gpu_ab_attn.sh VARIANT...)
set -eo pipefail
mkdir -p gpurun_out
for r in 1 2; do
  echo "== base $r"; timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
  for V in "$@"; do
    echo "== $V $r"; SAVQA_LIB=tools/ab/libsavqa_$V.so timeout -k 10 120 python -u tools/attn_bench.py --bf16 --B 512 2>&1 | grep -v amdgpu.ids
  done
done
for r in 1 2; do
  timeout -k 10 200 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base cfg3', d['value'])"
  for V in "$@"; do
    SAVQA_LIB=tools/ab/libsavqa_$V.so timeout -k 10 200 python -u bench.py --workload cfg3 --no-cpu-baseline --no-roofline | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$V cfg3', d['value'])"
  done
done
