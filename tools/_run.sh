set -o pipefail
cat /sys/fs/cgroup/cpu.max 2>&1; cat /sys/fs/cgroup/cpu.weight 2>&1; nproc; python3 -c "import os;print(len(os.sched_getaffinity(0)), os.cpu_count())"
for t in 16 64 256; do
timeout -k 5 60 python3 -c "
import torch,time
torch.set_num_threads($t)
a=torch.randn(2048,2048)
t0=time.perf_counter()
for _ in range(5): a@a
print($t, 'threads', (time.perf_counter()-t0)/5, 's per 2048^3 matmul')
" || echo "$t threads: timed out"
done
