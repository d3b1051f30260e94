#!/bin/bash
# Kernel trace of eager STF steps with the host out of the way (tools/gpu_critical.py:
# a spin kernel holds the GPU while the host enqueues each step), for critical-path analysis
set -e
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/stfspin
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/raw -o run -- python3 $root/tools/gpu_critical.py --model ${MODEL:-stf} --steps 3 --spin-ms ${SPIN:-40} > $out/crit.txt 2> $out/crit.err
f=$(find $out/raw -name 'run_kernel_trace.csv' | head -1)
cp $f $out/kernel_trace.csv
rm -rf $out/raw
gzip -f $out/kernel_trace.csv
