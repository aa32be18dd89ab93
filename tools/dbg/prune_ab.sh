set -e
bash tools/gpu.sh tests tests/test_model_gpu.py tests/test_blocks_gpu.py tests/test_fullsize_gpu.py tests/test_graph_capture_gpu.py tests/test_relation_gpu.py tests/test_longseq_gpu.py tests/test_train_gpu.py -k "not lowp"
for r in 1 2; do
  timeout -k 10 300 python -u tools/ab_flag.py PRUNE_L01=False --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('noprune', d['value'])"
  timeout -k 10 300 python -u tools/ab_flag.py PRUNE_L01=True --no-cpu-baseline --no-roofline 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print('prune', d['value'])"
done
