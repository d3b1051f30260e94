#!/bin/bash
# STF: halo kernel only when its persistent grid has >= STF_HALO_MIN_ITEMS items (A/B, one box)
set -e
out=gpurun_out/ab_items
mkdir -p $out
for v in 0 256 0 256; do
  STF_HALO_MIN_ITEMS=$v timeout -k 10 200 python3 bench.py --model stf --steps 30 --warmup 8 --no-cpu-baseline --no-dice --no-kernel-timer > $out/b$v.json 2> $out/b$v.err
  python3 -c "import json;d=json.load(open('$out/b$v.json'));print('items>=$v', d['value'], d['ms_per_step'])"
done
for v in 0 256; do
  STF_HALO_MIN_ITEMS=$v timeout -k 10 200 python3 tools/stf_shapes.py > $out/shapes$v.txt 2>&1
  tail -1 $out/shapes$v.txt
done
