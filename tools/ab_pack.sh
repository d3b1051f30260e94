set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu > gpurun_out/kt.log 2>&1
for m in unet stf; do
  STF_PACK_TILED=0 timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > gpurun_out/ab_${m}_0.json 2>/dev/null
  STF_PACK_TILED=1 timeout -k 10 300 python bench.py --model $m --no-cpu-baseline > gpurun_out/ab_${m}_1.json 2>/dev/null
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1
grep -i pack $GRAFT_REPO_ROOT/gpurun_out/pp/run_kernel_stats.csv
