set -eo pipefail
bash tools/gpu.sh prof r04 cfg2 cfg3 cfg4 cfg5 rel
TO=400 bash tools/gpu.sh bench cfg2 cfg3 cfg4 cfg5 rel
