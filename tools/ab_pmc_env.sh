#!/bin/bash
# A/B an environment toggle on the UNet bench (2 interleaved rounds) plus one FETCH_SIZE
# pass per value (HBM reads per kernel):  VAR=NAME VALUES="0 1" bash tools/ab_pmc_env.sh
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VALUES:-0 1}; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-dice > gpurun_out/abp_$v.json 2> gpurun_out/abp_$v.err || { tail gpurun_out/abp_$v.err; exit 1; }
    python3 - "$VAR=$v" gpurun_out/abp_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = d["kernels_census_step"]
top = sorted(ks.items(), key=lambda kv: -kv[1]["ms"])[:4]
print(sys.argv[1], f"{d['value']:.1f}/s {d['ms_per_step']:.2f} ms |", " | ".join(f"{k[:26]} {v['ms']:.3f}" for k, v in top))
PY
  done
done
for v in ${VALUES:-0 1}; do
  ( cd /tmp && export TMPDIR=/tmp && env $VAR=$v timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/abp_pmc_$v/FETCH_SIZE" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-kernel-timer --no-dice --steps 3 --warmup 1 > /dev/null 2>&1 ) || exit 1
  python3 - "$VAR=$v" gpurun_out/abp_pmc_$v/FETCH_SIZE/run_results.db <<'PY'
import sqlite3, sys, re
from collections import defaultdict
agg = defaultdict(lambda: [0, 0.0])
for name, val in sqlite3.connect(sys.argv[2]).execute("select name, counter_value from pmc_events where counter_name='FETCH_SIZE'"):
    n = re.sub(r"\(anonymous namespace\)::|^void ", "", name); n = n[: n.find(">(") + 1] if ">(" in n else n.split("(")[0]
    agg[n][0] += 1; agg[n][1] += float(val)
for k, (c, v) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:5]:
    print(sys.argv[1], f"{2 * v * 1024 / c / 1e6:9.1f} MB fetched/launch x{c} {k}")
PY
  rm -rf gpurun_out/abp_pmc_$v
done
