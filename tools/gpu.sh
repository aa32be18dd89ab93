#!/bin/bash
# One parameterised entry point for every GPU-box job of this repo (run through gpurun).
# Every GPU step runs under its own time limit, steps are chained with && (set -e), and the
# script stops at the first failing step.
#
#   bash tools/gpu.sh suite                   full `pytest -m gpu` + smoke + default bench line
#   bash tools/gpu.sh tests PATH... [-k EXPR] selected GPU tests (pytest args passed through)
#   bash tools/gpu.sh bench [WORKLOAD...]     bench lines (default: cfg2), JSON in gpurun_out/
#   bash tools/gpu.sh prof TAG [WORKLOAD...]  rocprof kernel stats + FETCH/WRITE PMC passes
#                                             (tools/profile_round.sh) per workload
#   bash tools/gpu.sh gemm [LAYOUT:M:N:K...]  savqa_gemm vs torch.mm on the cfg-2 shapes
#   bash tools/gpu.sh lp [ARGS...]            tools/lp_bench.py (bf16 / fp8 GEMM shapes)
#   bash tools/gpu.sh attn [ARGS...]          tools/attn_bench.py
#   bash tools/gpu.sh ab VARIANT... [-- CMD]  interleaved A/B of variant libraries
#                                             tools/ab/libsavqa_VARIANT.so (SAVQA_LIB) against the
#                                             in-tree one: CMD (default: the cfg-2 GEMM bench),
#                                             then the cfg-2 bench line; WL=cfg3 picks the workload
#   bash tools/gpu.sh lpdiag                  lp diagnostic builds + SQ PMC passes (tools/lp_pmc.sh)
set -eo pipefail
mkdir -p gpurun_out
cmd=${1:-suite}
shift || true
TO=${TO:-300}

quiet() { grep -v amdgpu.ids || true; }

bench_line() {  # bench_line WORKLOAD [extra bench.py args]
  local w=$1; shift
  timeout -k 10 ${TO} python -u bench.py --workload "$w" "$@" > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err \
    || { tail -20 gpurun_out/bench_$w.err; return 1; }
  python -c "import json;d=json.load(open('gpurun_out/bench_$w.json'));r=d.get('roofline') or {};print('$w', d['value'], d['unit'], d['ms_per_step'], 'ms/step', r.get('kernel'), r.get('frac'))"
}

case "$cmd" in
  suite)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
      > gpurun_out/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
    tail -3 gpurun_out/pytest_gpu.log
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { tail -20 gpurun_out/smoke.log; exit 1; }
    tail -2 gpurun_out/smoke.log
    bench_line cfg2
    ;;
  tests)
    timeout -k 10 ${TO} python -u -m pytest -x -v --timeout 280 --timeout-method thread "$@" \
      > gpurun_out/tests.log 2>&1 || { grep -E "FAILED|Error" gpurun_out/tests.log | head -20; tail -60 gpurun_out/tests.log; exit 1; }
    grep -E "PASSED|SKIPPED|XFAIL" gpurun_out/tests.log | tail -40
    tail -2 gpurun_out/tests.log
    ;;
  bench)
    for w in ${@:-cfg2}; do
      if [ "$w" = cfg2 ]; then bench_line cfg2; else bench_line "$w" --no-cpu-baseline; fi
    done
    ;;
  prof)
    tag=${1:-r03}; shift || true
    for w in ${@:-cfg2}; do
      timeout -k 10 600 bash tools/profile_round.sh "$tag" "$w"
    done
    ;;
  gemm)
    timeout -k 10 ${TO} python -u tools/gemm_bench.py "$@" 2>&1 | quiet
    ;;
  lp)
    timeout -k 10 ${TO} python -u tools/lp_bench.py "$@" 2>&1 | quiet
    ;;
  attn)
    timeout -k 10 ${TO} python -u tools/attn_bench.py "$@" 2>&1 | quiet
    ;;
  ab)
    vs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do vs+=("$1"); shift; done
    [ "${1:-}" = "--" ] && shift
    run=("$@"); [ ${#run[@]} -eq 0 ] && run=(python -u tools/gemm_bench.py)
    wl=${WL:-cfg2}
    for r in 1 2; do
      echo "== base $r"; timeout -k 10 ${TO} "${run[@]}" 2>&1 | quiet
      for v in "${vs[@]}"; do
        echo "== $v $r"; SAVQA_LIB=tools/ab/libsavqa_$v.so timeout -k 10 ${TO} "${run[@]}" 2>&1 | quiet
      done
    done
    for r in 1 2; do
      timeout -k 10 ${TO} python -u bench.py --workload $wl --no-cpu-baseline --no-roofline \
        | python -c "import json,sys;d=json.loads(sys.stdin.read());print('base $wl', d['value'])"
      for v in "${vs[@]}"; do
        SAVQA_LIB=tools/ab/libsavqa_$v.so timeout -k 10 ${TO} python -u bench.py --workload $wl --no-cpu-baseline --no-roofline \
          | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$v $wl', d['value'])"
      done
    done
    ;;
  lpdiag)
    timeout -k 10 ${TO} python -u tools/lp_bench.py --dbg1 > gpurun_out/lp_dbg1.log 2>&1 || { tail -20 gpurun_out/lp_dbg1.log; exit 1; }
    quiet < gpurun_out/lp_dbg1.log
    bash tools/lp_pmc.sh NT 37376 2048 512 bf16 1 ffn1
    bash tools/lp_pmc.sh TN 2048 512 37376 atomic 0 dwffn1
    python tools/pmc_table.py gpurun_out/pmc | tee gpurun_out/lp_pmc_table.txt
    ;;
  *)
    echo "unknown command $cmd"; exit 2
    ;;
esac
