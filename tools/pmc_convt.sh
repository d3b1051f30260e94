#!/bin/bash
# PMC passes (traffic, instruction mix) over tools/convt_cfg.py: one rocprofv3 run per pass.
set -e
out=$GRAFT_REPO_ROOT/gpurun_out/pmc_convt
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d "$out/p$i" -o run -- \
    python3 "$GRAFT_REPO_ROOT/tools/convt_cfg.py" 64 > "$out/p$i.log" 2>&1
done
