#!/bin/bash
# UNet weight gradients inline vs on a side stream (1 or 2 workgroups per CU), same box
mkdir -p gpurun_out/abside
for rep in 1 2; do
  for cfg in "0 256" "1 256" "1 512" "1 384"; do
    set -- $cfg
    STF_UNET_WGRAD_SIDE=$1 STF_SIDE_WGRAD_BLOCKS=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/abside/b_$1_$2_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/abside/b_$1_$2_$rep.json "side=$1 blocks=$2 rep=$rep"
  done
done
