#!/bin/bash
# Same-box STF A/B: the in-tree library vs stf-unet_amd/stfunet/libstfunet_hip_alt.so
#   bash tools/ab_stf.sh [reps]
set -o pipefail
alt=$GRAFT_REPO_ROOT/stf-unet_amd/stfunet/libstfunet_hip_alt.so
for rep in $(seq ${1:-3}); do
  for v in alt new; do
    if [ $v = alt ]; then export STF_LIB=$alt; else unset STF_LIB; fi
    timeout -k 10 300 python bench.py --model stf --no-cpu-baseline > gpurun_out/abstf_$v.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/abstf_$v.json'));print('$v', d['value'], d['ms_per_step'])"
  done
done
unset STF_LIB
