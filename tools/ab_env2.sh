#!/bin/bash
# Same-box A/B of one environment switch on a bench command, interleaved:
#   bash tools/ab_env2.sh "<VAR=a>" "<VAR=b>" reps  <bench args...>
a=$1; b=$2; reps=$3; shift 3
mkdir -p gpurun_out
for r in $(seq $reps); do
  for v in "$a" "$b"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-dice "$@" > gpurun_out/abenv.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abenv.json').read().strip().splitlines()[-1]); print(sys.argv[1], d['config']['workload'][:18], d['value'], d['ms_per_step'])" "$v"
  done
done
