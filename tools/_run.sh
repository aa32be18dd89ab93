set -eo pipefail
bash tools/gpu.sh suite > gpurun_out/suite.txt 2>&1 || { tail -30 gpurun_out/suite.txt; exit 1; }
cat gpurun_out/suite.txt
