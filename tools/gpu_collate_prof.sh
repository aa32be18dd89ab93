set -e
mkdir -p gpurun_out/collate_prof
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/collate_prof -o run -- python3 -u tools/collate_bench.py > gpurun_out/collate_prof.log 2>&1 || { tail -30 gpurun_out/collate_prof.log; exit 1; }
cat gpurun_out/collate_prof.log | grep workload
find gpurun_out/collate_prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/collate_prof -name "*kernel_stats.csv" | head -1); grep -i "collate\|Name" "$f" | cut -c1-200
