#!/bin/bash
# Same-box A/B of host-side (Python) changes: the baseline package tree in abpkg/
# (git archive of the old commit + the built .so files) vs the working tree.
mkdir -p gpurun_out/abhost
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export STF_PKG_ROOT=$GRAFT_REPO_ROOT/abpkg/stf-unet_amd; else unset STF_PKG_ROOT; fi
    timeout -k 10 200 python tools/host_breakdown.py --model ${MODEL:-stf} > gpurun_out/abhost/hb_${v}_$rep.txt 2>&1 || { tail gpurun_out/abhost/hb_${v}_$rep.txt; exit 1; }
    echo "$v rep $rep: $(tail -n 1 gpurun_out/abhost/hb_${v}_$rep.txt)"
  done
done
unset STF_PKG_ROOT
