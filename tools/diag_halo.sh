#!/bin/bash
# Ablations of the halo conv kernel on the cfg2 layer shapes (STF_HALO_DIAG):
# 0 = real, 1 = no output stores, 2 = no reloads after the first stage, 3 = no MFMA/LDS reads
mkdir -p gpurun_out
for d in ${DIAGS:-0 1 2 3}; do
  STF_HALO_DIAG=$d timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/diag_$d.log 2>&1 || exit 1
  echo "== diag $d"; grep -E "^(enc1.3|enc2.3|dec1.0|dec2.0|enc3.3|dec1.3|TOTAL)" gpurun_out/diag_$d.log | cut -c1-120
done
