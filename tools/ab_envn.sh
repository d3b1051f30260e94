#!/bin/bash
# Same-box comparison of N environment settings on one bench command, interleaved:
#   bash tools/ab_envn.sh reps "<A=1 B=2>" "<A=0>" ... -- <bench args...>
reps=$1; shift
envs=()
while [ "$1" != "--" ]; do envs+=("$1"); shift; done
shift
mkdir -p gpurun_out
for r in $(seq $reps); do
  for v in "${envs[@]}"; do
    env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-dice "$@" > gpurun_out/abenv.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/abenv.json').read().strip().splitlines()[-1]); print(sys.argv[1].ljust(40), d['config']['workload'][:18], d['value'], d['ms_per_step'])" "$v"
  done
done
