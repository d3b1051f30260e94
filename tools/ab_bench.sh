#!/bin/bash
# A/B an environment toggle on whole-step benches (both models), after the GPU tests:
#   VAR=NAME VALUES="0 1" bash tools/ab_bench.sh
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
for rep in 1 2; do
  for v in ${VALUES:-0 1}; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/abb_unet_$v.json 2> gpurun_out/abb_unet_$v.err || { tail gpurun_out/abb_unet_$v.err; exit 1; }
    env $VAR=$v timeout -k 10 300 python bench.py --model stf --no-cpu-baseline > gpurun_out/abb_stf_$v.json 2> gpurun_out/abb_stf_$v.err || { tail gpurun_out/abb_stf_$v.err; exit 1; }
    python - "$VAR=$v" gpurun_out/abb_unet_$v.json gpurun_out/abb_stf_$v.json <<'PY'
import json, sys
out = [sys.argv[1]]
for f in sys.argv[2:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    out.append(f"{d['config']['workload']}: {d['value']:.1f} {d['unit']} {d['ms_per_step']:.2f} ms")
print(" | ".join(out))
PY
  done
done
