#!/bin/bash
# Round profile of a bench.py workload (run on the GPU box via gpurun):
#   1. rocprofv3 --kernel-trace --stats          -> kernel durations (+ bench JSON line)
#   2. rocprofv3 --pmc FETCH_SIZE  (own pass)     -> HBM read bytes
#   3. rocprofv3 --pmc WRITE_SIZE  (own pass)     -> HBM write bytes
# then tools/summarize_prof.py writes gpurun_out/prof_<tag>_<wl>/<tag>_<wl>_{kernel_stats.csv,roofline.json}
# (copied into profiles/ by hand after the gpurun call; bench.py reads the committed
# roofline.json for its `traffic` field).
# usage: bash tools/profile_round.sh TAG WORKLOAD   (e.g. r02 cfg2)
set -e
TAG=${1:-r02}
WL=${2:-cfg2}
STEPS=${STEPS:-5}
O=gpurun_out/prof_${TAG}_${WL}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python bench.py --workload $WL --steps $STEPS --warmup 2 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- $CMD > $O/bench_trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $CMD > $O/bench_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- $CMD > $O/bench_write.log 2>&1
LPS=$(grep '^{"metric"' $O/bench_trace.log | python -c 'import json,sys; r=json.loads(sys.stdin.read())["roofline"]; print(json.dumps({r["kernel"]: r["launches_per_step"]}))')
python tools/summarize_prof.py $O/trace $O/fetch $O/write $O/${TAG}_${WL} "$LPS" > $O/summary.log 2>&1
grep '^{"metric"' $O/bench_trace.log > $O/${TAG}_${WL}_bench_line_under_rocprof.json
echo "profile $WL done"
