#!/bin/bash
# Kernel trace of plan-replayed training steps (bench.py, native plans: the host runs ahead
# of the GPU, so the trace shows the GPU's own critical path); analyse with
#   python tools/crit_path.py gpurun_out/trace_<tag>/kernel_trace.csv.gz
#   bash tools/stf_trace_plan.sh <tag> <bench args...>
set -e
root=$GRAFT_REPO_ROOT
tag=$1; shift
out=$root/gpurun_out/trace_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/raw -o run -- python3 $root/bench.py --no-dice --no-cpu-baseline --no-kernel-timer --steps 4 --warmup 3 "$@" > $out/bench.json 2> $out/bench.err
f=$(find $out/raw -name 'run_kernel_trace.csv' | head -1)
cp $f $out/kernel_trace.csv
rm -rf $out/raw
gzip -f $out/kernel_trace.csv
