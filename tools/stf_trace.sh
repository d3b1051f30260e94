set -e
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/stftrace
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/raw -o run -- python3 $root/bench.py --model stf --steps 10 --warmup 5 --no-cpu-baseline --no-dice $STF_TRACE_ARGS > $out/bench.json 2> $out/bench.err
f=$(find $out/raw -name 'run_kernel_trace.csv' | head -1)
cp $f $out/kernel_trace.csv
rm -rf $out/raw
cd $root
python3 tools/trace_gaps.py $out/kernel_trace.csv --steps 5 --top 25 > $out/gaps.txt
gzip $out/kernel_trace.csv
