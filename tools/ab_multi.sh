#!/bin/bash
# Same-box A/B of several builds of the HIP library, interleaved: per build directory (each holding
# a libstfunet_hip.so; "tree" = the in-tree build) the UNet layer bench (tools/bench_layers.py:
# fwd / dgrad / wgrad totals) and the default bench line.
#   bash tools/ab_multi.sh REPS DIR1 DIR2 ...     e.g.  bash tools/ab_multi.sh 2 abbase tree abvar_E
set -o pipefail
reps=$1; shift
mkdir -p gpurun_out
for rep in $(seq $reps); do
  for d in "$@"; do
    if [ "$d" = tree ]; then unset STF_LIB; else export STF_LIB=$GRAFT_REPO_ROOT/$d/libstfunet_hip.so; fi
    timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/abm_layers.log 2>&1 || { tail gpurun_out/abm_layers.log; exit 1; }
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-dice ${BENCH_ARGS} > gpurun_out/abm_bench.json 2>/dev/null || exit 1
    python3 - "$d" gpurun_out/abm_bench.json gpurun_out/abm_layers.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
tot = [l.strip() for l in open(sys.argv[3]) if l.startswith("TOTAL ") and "convT" not in l]
print(f"{sys.argv[1]:8s} {d['value']:8.1f}/s {d['ms_per_step']:6.2f} ms | " + " | ".join(tot), flush=True)
PY
  done
done
unset STF_LIB
