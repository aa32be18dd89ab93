set -e
SAVQA_LIB=structured-alignment-vqa_amd/csrc/build/libsavqa_skip2.so timeout -k 10 100 python tools/attn_bench.py > gpurun_out/at4.log 2>&1
