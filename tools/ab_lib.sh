#!/bin/bash
# Same-box A/B of two builds of the HIP library (box-to-box spread is ~5 %, larger
# than most kernel changes): the baseline build is saved with
#   mkdir -p abbase && cp stf-unet_amd/stfunet/libstfunet_hip.so abbase/   (before the change)
# and this script runs the layer bench and both model benches, alternating builds.
#   bash tools/ab_lib.sh [reps]
set -o pipefail
mkdir -p gpurun_out
base=$GRAFT_REPO_ROOT/abbase/libstfunet_hip.so
[ -f "$base" ] || { echo "no baseline build at $base"; exit 1; }
for rep in $(seq ${1:-2}); do
  for v in base new; do
    if [ $v = base ]; then export STF_LIB=$base; else unset STF_LIB; fi
    timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/ablib_layers_$v.log 2>&1 || { tail gpurun_out/ablib_layers_$v.log; exit 1; }
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ablib_unet_$v.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --model stf --no-cpu-baseline > gpurun_out/ablib_stf_$v.json 2>/dev/null || exit 1
    python3 - $v gpurun_out/ablib_unet_$v.json gpurun_out/ablib_stf_$v.json gpurun_out/ablib_layers_$v.log <<'PY'
import json, sys
out = [sys.argv[1]]
for f in sys.argv[2:4]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    out.append(f"{d['config']['workload'][:14]}: {d['value']:.1f}/s {d['ms_per_step']:.2f} ms")
out += [l.strip() for l in open(sys.argv[4]) if l.startswith("TOTAL ") and "convT" not in l]
print(" | ".join(out))
PY
  done
done
unset STF_LIB
