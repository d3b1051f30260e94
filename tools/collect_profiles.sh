#!/bin/bash
# Round profile collection (run on the GPU box from the repo root):
#   kernel-trace stats for the UNet (cfg2) and STF (cfg3) bench steps, and the
#   two PMC passes (HBM traffic) for cfg2.  Outputs under gpurun_out/prof_<tag>.
set -e
tag=${1:-r01}
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/unet" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$out/unet.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$out/stf" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --model stf --steps 10 --warmup 3 --no-cpu-baseline > "$GRAFT_REPO_ROOT/$out/stf.log" 2>&1
cd "$GRAFT_REPO_ROOT"
bash tools/pmc_passes.sh $out/pmc --steps 3 --warmup 1
