set -eo pipefail
bash tools/gpu.sh suite > gpurun_out/suite.txt 2>&1 || { tail -30 gpurun_out/suite.txt; exit 1; }
cat gpurun_out/suite.txt
TO=400 bash tools/gpu.sh bench cfg3 cfg5 > gpurun_out/bench35.txt 2>&1 || { tail -20 gpurun_out/bench35.txt; exit 1; }
cat gpurun_out/bench35.txt
