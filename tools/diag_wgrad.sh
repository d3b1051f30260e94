#!/bin/bash
# Ablations of wgrad3x3 (STF_WGRAD_DIAG): 0 = real, 1 = no global loads after the first step, 2 = no MFMA/LDS reads
mkdir -p gpurun_out
for d in 0 1 2; do
  STF_WGRAD_DIAG=$d timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/wd_$d.log 2>&1 || exit 1
  echo "== diag $d"; grep -E "^(enc1.3|enc2.3|enc3.3|dec2.0|dec1.0|TOTAL wgrad)" gpurun_out/wd_$d.log | awk '{print $1, $(NF-3), $(NF-2), $(NF-1), $NF}'
done
