#!/bin/bash
# Instruction mix per kernel of one bench run (one rocprofv3 --pmc pass, kernel trace only):
# VALU issue time vs duration finds VALU-bound memory kernels (tools/pmc_mix_summary.py).
# Usage: bash tools/pmc_mix.sh OUTDIR [bench args...]
set -e
out=$GRAFT_REPO_ROOT/$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES --kernel-trace -d "$out" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-kernel-timer --no-dice --steps 3 --warmup 2 "$@" > "$out/bench.log" 2>&1
