# A/B of the backward stack schedule (SAVQA_BWD_ORDER): phase finish times at N=1
set -e
mkdir -p gpurun_out
for o in concurrent dec enc4 enc2 syb_first; do
  SAVQA_BWD_ORDER=$o timeout -k 10 240 python -u tools/tail_probe.py > gpurun_out/tail_$o.json 2> gpurun_out/tail_$o.err
  cat gpurun_out/tail_$o.json
done
