#!/bin/bash
# STF cfg3: eager vs HIP-graph replay of the whole training step, same box, interleaved
mkdir -p gpurun_out/abgraph
for rep in 1 2; do
  for g in off on; do
    timeout -k 10 300 python bench.py --model stf --no-cpu-baseline --graph $g > gpurun_out/abgraph/stf_${g}_$rep.json 2>gpurun_out/abgraph/stf_${g}_$rep.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d.get('execution'))" gpurun_out/abgraph/stf_${g}_$rep.json "graph=$g rep=$rep"
  done
done
