set -eo pipefail
SEED=0 timeout -k 10 600 python -u tools/x6_audit.py 2>&1 | grep -v amdgpu.ids > gpurun_out/x6_audit_r05.txt
head -30 gpurun_out/x6_audit_r05.txt
