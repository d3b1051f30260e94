#!/bin/bash
# STF encoder layer shapes (128 images) per forced linear tile config, split-K on/off (one box)
set -e
out=gpurun_out/ab_stf_layers2
mkdir -p $out
for c in auto B C A E; do
  if [ $c = auto ]; then e="STF_AB=0"; else e="STF_IGEMM_CFG=$c"; fi
  env $e timeout -k 10 200 python3 tools/bench_layers.py --stf > $out/$c.txt 2>&1
  echo "== $c"; grep "^l\|TOTAL" $out/$c.txt
done
STF_SPLITK=0 timeout -k 10 200 python3 tools/bench_layers.py --stf > $out/nosplit.txt 2>&1
echo "== auto, no split-K"; grep "^l\|TOTAL" $out/nosplit.txt
