#!/bin/bash
# Round profile of the judged bench command (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats          -> kernel durations (+ bench JSON line)
#   2. rocprofv3 --pmc FETCH_SIZE  (own pass)     -> HBM read bytes
#   3. rocprofv3 --pmc WRITE_SIZE  (own pass)     -> HBM write bytes
# then tools/summarize_prof.py writes gpurun_out/prof_<tag>/<tag>_bench_{kernel_stats.csv,roofline.json}
# (copied into profiles/ by hand after the gpurun call).
set -e
TAG=${1:-r01}
STEPS=${STEPS:-5}
O=gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python bench.py --steps $STEPS --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O/bench_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD > $O/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD > $O/bench_write.log 2>&1
LPS=$(grep '^{"metric"' $O/bench_trace.log | python -c 'import json,sys; r=json.loads(sys.stdin.read())["roofline"]; print(json.dumps({r["kernel"]: r["launches_per_step"]}))')
python tools/summarize_prof.py $O/trace $O/fetch $O/write $O/${TAG}_bench "$LPS" > $O/summary.log 2>&1
grep '^{"metric"' $O/bench_trace.log > $O/${TAG}_bench_line_under_rocprof.json
# (only gpurun_out/ comes back from the box: copy $O/${TAG}_bench* into profiles/ afterwards)
echo done
