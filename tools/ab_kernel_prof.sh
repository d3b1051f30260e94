#!/bin/bash
# Same-box kernel-level A/B of two library builds under rocprofv3 --kernel-trace --stats:
# the baseline build in abbase/ (STF_LIB) vs the working tree's, bench.py [ARGS], and the
# per-kernel averages of the kernels matching $KPAT side by side.
#   KPAT="wgrad_reduce|pack_tiled" bash tools/ab_kernel_prof.sh [bench args]
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/abprof
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  if [ $v = base ]; then export STF_LIB=$root/abbase/libstfunet_hip.so; else unset STF_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/$v -o run -- \
    python3 $root/bench.py --no-cpu-baseline --steps 10 --warmup 3 "$@" > $out/bench_$v.json 2> $out/$v.log || exit 1
done
unset STF_LIB
python3 - $out "${KPAT:-wgrad_reduce}" <<'PY'
import csv, glob, json, re, sys
out, pat = sys.argv[1], re.compile(sys.argv[2])
for v in ("base", "new"):
    f = glob.glob(f"{out}/{v}/**/run_kernel_stats.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if pat.search(r["Name"])]
    d = json.loads(open(f"{out}/bench_{v}.json").read().strip().splitlines()[-1])
    print(v, f"{d['value']:.1f}/s", " | ".join(f"{r['Name'][:40]} n={r['Calls']} avg={float(r['AverageNs'])/1e3:.1f}us" for r in rows))
PY
