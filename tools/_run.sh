set -eo pipefail
bash tools/gpu.sh suite -s > gpurun_out/suite.txt 2>&1 || { tail -30 gpurun_out/suite.txt; exit 1; }
tail -4 gpurun_out/suite.txt
grep "per-gradient worst" gpurun_out/pytest_gpu.log | cut -c1-1500
