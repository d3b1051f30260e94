#!/bin/bash
# STF cfg3: workgroups of the side-stream fused weight gradients (STF_SIDE_WGRAD_BLOCKS), one box
set -e
out=gpurun_out/ab_sideblocks
mkdir -p $out
for r in 1 2; do
for v in 256 384 192 320; do
  STF_SIDE_WGRAD_BLOCKS=$v timeout -k 10 200 python3 bench.py --model stf --steps 30 --warmup 8 --no-cpu-baseline --no-dice --no-kernel-timer > $out/b$v.json 2> $out/b$v.err
  python3 -c "import json;d=json.load(open('$out/b$v.json'));print('blocks $v', d['value'], d['ms_per_step'])"
done
done
