# Round-end profiles: rocprof kernel stats + FETCH/WRITE PMC passes of the cfg2 / cfg3 / cfg5
# bench commands (tools/profile_round.sh), each step under its own limit
set -eo pipefail
for w in ${WORKLOADS:-cfg2 cfg3 cfg5}; do
  timeout -k 10 500 bash tools/profile_round.sh r02 $w
done
