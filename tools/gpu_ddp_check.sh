# DDP path checks on one GPU: DDP GPU tests (2 gloo ranks share the card), a 2-rank gloo
# rehearsal of bench.py's N>1 path (row-sparse tables + gated backward schedule), N=1 bench
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ddp_gpu.log 2>&1 || { tail -30 gpurun_out/ddp_gpu.log; exit 1; }
tail -3 gpurun_out/ddp_gpu.log
SAVQA_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
  --no-cpu-baseline --no-roofline > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err
cat gpurun_out/bench_gloo2.json
timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err
cat gpurun_out/bench_n1.json
