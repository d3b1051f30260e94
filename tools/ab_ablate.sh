#!/bin/bash
# Interleaved same-box runs of tools/ablate_bench.py: bash tools/ab_ablate.sh reps "none bn1 ..." [bench args]
reps=$1; shift
abl=$1; shift
mkdir -p gpurun_out
for r in $(seq $reps); do
  for a in $abl; do
    timeout -k 10 300 python tools/ablate_bench.py $a --no-cpu-baseline --no-dice "$@" > gpurun_out/ablate.json 2>gpurun_out/ablate.err || { tail -5 gpurun_out/ablate.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ablate.json').read().strip().splitlines()[-1]); print(sys.argv[1].ljust(12), d['config']['workload'][:18], d['value'], d['ms_per_step'])" "$a"
  done
done
