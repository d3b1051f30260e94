#!/bin/bash
# STF cfg3 step: eager vs HIP-graph replay under the runtime's graph knobs (one box).
#   bash tools/ab_graph.sh
set -e
out=gpurun_out/ab_graph
mkdir -p $out
run() {  # tag "ENV=.. ENV=.." "bench args"
  tag=$1
  timeout -k 10 200 env $2 python3 bench.py --model stf --steps 30 --warmup 8 --no-cpu-baseline --no-dice \
    --no-kernel-timer $3 > $out/$tag.json 2> $out/$tag.err
  python3 -c "import json;d=json.load(open('$out/$tag.json'));print('$tag', d['value'], d['ms_per_step'], d['execution'])"
}
run eager "STF_AB=0" "--graph off"
run graph "STF_AB=0" "--graph on"
run eager2 "STF_AB=0" "--graph off"
run graph2 "STF_AB=0" "--graph on"
