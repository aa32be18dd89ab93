set -eo pipefail
timeout -k 10 900 bash tools/profile_round.sh r04 cfg5
ls gpurun_out/prof_r04_cfg5/
