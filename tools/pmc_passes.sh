#!/bin/bash
# HBM traffic per kernel (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc passes (they do not fit one pass), kernel trace only.
# Usage: bash tools/pmc_passes.sh OUTDIR [bench args...]
set -e
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 500 rocprofv3 --pmc $c --kernel-trace -d "$GRAFT_REPO_ROOT/$out/$c" -o run -- \
    python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-kernel-timer --no-dice "$@" > "$GRAFT_REPO_ROOT/$out/$c.log" 2>&1
done
