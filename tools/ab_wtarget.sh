#!/bin/bash
# weight gradients inline vs on a side stream (one workgroup per CU there), STF + UNet, one box
set -e
out=gpurun_out/ab_wtarget
mkdir -p $out
run() {  # tag "ENV=.." "args"
  timeout -k 10 200 env $2 python3 bench.py $3 --steps 30 --warmup 8 --no-cpu-baseline --no-dice \
    --no-kernel-timer > $out/$1.json 2> $out/$1.err
  python3 -c "import json;d=json.load(open('$out/$1.json'));print('$1 $2 $3', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
run stf "STF_AB=0" "--model stf"
run stf_inline "STF_WGRAD_SIDE=0" "--model stf"
run unet "STF_AB=0" ""
run unet_side "STF_UNET_WGRAD_SIDE=1" ""
done
