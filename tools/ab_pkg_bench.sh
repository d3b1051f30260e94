#!/bin/bash
# Same-box A/B of host-side (Python) changes on both benches: the package tree in abpkg/
# (git archive of the baseline commit + the built .so files) vs the working tree.
mkdir -p gpurun_out/abpkg
for rep in ${REPS:-1 2}; do
  for v in base new; do
    if [ $v = base ]; then export STF_PKG_ROOT=$GRAFT_REPO_ROOT/abpkg/stf-unet_amd; else unset STF_PKG_ROOT; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/abpkg/u_${v}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --model stf --no-cpu-baseline --steps 30 --warmup 5 > gpurun_out/abpkg/s_${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "
import json,sys
out=[]
for f in sys.argv[2:]:
    d=json.loads(open(f).read().strip().splitlines()[-1]); out.append('%s %.1f %.2f' % (d['config']['workload'][:5], d['value'], d['ms_per_step']))
print(sys.argv[1], ' | '.join(out))" "$v rep $rep" gpurun_out/abpkg/u_${v}_$rep.json gpurun_out/abpkg/s_${v}_$rep.json
  done
done
