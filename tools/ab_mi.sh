set -e
for v in mi32 mi16; do echo "== $v"; SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so timeout -k 10 150 python -u tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | awk '{print $1, $2, $8, $9, $10}'; done
SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_mi16.so timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_blocks_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
for v in mi32 mi16; do echo "== bench $v"; SAVQA_LIB=structured-alignment-vqa_amd/csrc/variants/libsavqa_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline 2>&1 | tail -1 | cut -c1-200; done
