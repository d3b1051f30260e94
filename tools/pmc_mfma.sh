#!/bin/bash
# MFMA utilisation per kernel (MI355X_MICROARCH.md 'rocprofv3 PMC slots'): one rocprofv3
# --pmc pass with SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_BF16 and
# GRBM_GUI_ACTIVE (2 SQ + 1 GRBM counters: fits one pass), kernel trace only.
# Usage: bash tools/pmc_mfma.sh OUTDIR [bench args...]
set -e
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE \
  --kernel-trace -d "$GRAFT_REPO_ROOT/$out/MFMA" -o run -- \
  python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-kernel-timer --no-dice "$@" > "$GRAFT_REPO_ROOT/$out/MFMA.log" 2>&1
