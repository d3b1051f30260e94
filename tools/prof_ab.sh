#!/bin/bash
# Kernel-trace A/B of an environment toggle on one bench config (GPU box, repo root):
#   VAR=NAME VALUES="0 1" ARGS="--model stf" bash tools/prof_ab.sh
# Per-kernel per-step table for each value side by side (tools/prof_diff.py).
set -o pipefail
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/prof_ab
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in ${VALUES:-0 1}; do
  export $VAR=$v
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/v$v -o run -- \
    python3 $root/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timer $ARGS > $out/v$v.log 2>&1 || { tail $out/v$v.log; exit 1; }
done
cd $root
python3 tools/prof_diff.py --steps 14 $(for v in ${VALUES:-0 1}; do ls $out/v$v/*kernel_stats.csv | head -1; done)
