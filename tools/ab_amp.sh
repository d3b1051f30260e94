#!/bin/bash
# fp16 (--amp) steps: AdamW taking GradScaler's device scale / inf flag vs the scaler's
# unscale_ + host inf check (STF_AMP_DEVICE_STEP=0), same box, interleaved
mkdir -p gpurun_out/abamp
for rep in 1 2; do
  for v in 0 1; do
    STF_AMP_DEVICE_STEP=$v timeout -k 10 300 python bench.py --dtype fp16 --no-cpu-baseline > gpurun_out/abamp/unet_${v}_$rep.json 2>/dev/null || exit 1
    STF_AMP_DEVICE_STEP=$v timeout -k 10 300 python bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abamp/cfg5_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys
for f in sys.argv[2:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); print(sys.argv[1], d['config']['workload'][:16], d['value'], d['ms_per_step'])" "device_step=$v rep=$rep" gpurun_out/abamp/unet_${v}_$rep.json gpurun_out/abamp/cfg5_${v}_$rep.json
  done
done
