#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench command; the stats csv lands in gpurun_out/<tag>_stats.csv
#   bash tools/prof_stats.sh <tag> <bench args...>
tag=$1; shift
root=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/gpurun_out/prof_$tag -o run -- \
  python3 $root/bench.py --no-cpu-baseline --no-dice "$@" > $root/gpurun_out/${tag}_bench.json 2> $root/gpurun_out/${tag}.log || exit 1
cd $root
cp $(find gpurun_out/prof_$tag -name run_kernel_stats.csv | head -1) gpurun_out/${tag}_stats.csv
gzip -c $(find gpurun_out/prof_$tag -name run_kernel_trace.csv | head -1) > gpurun_out/${tag}_trace.csv.gz
rm -rf gpurun_out/prof_$tag
