#!/bin/bash
# SQ counters for one conv layer kernel (tools/one_layer.py), two passes of <= 8 SQ counters.
# Usage: bash tools/pmc_layer.sh OUT fwd 256 64 64
set -e
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVES --kernel-trace -d "$GRAFT_REPO_ROOT/$out/p1" -o run -- python3 "$GRAFT_REPO_ROOT/tools/one_layer.py" "$@" > "$GRAFT_REPO_ROOT/$out/p1.log" 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL --kernel-trace -d "$GRAFT_REPO_ROOT/$out/p2" -o run -- python3 "$GRAFT_REPO_ROOT/tools/one_layer.py" "$@" > "$GRAFT_REPO_ROOT/$out/p2.log" 2>&1
