#!/bin/bash
# STF encoder conv shapes under each implicit-GEMM tile configuration
mkdir -p gpurun_out
for c in ${CFGS:-0 A B C D}; do
  STF_IGEMM_CFG=$c timeout -k 10 200 python tools/bench_layers.py --stf > gpurun_out/ls_$c.log 2>&1 || { tail -5 gpurun_out/ls_$c.log; exit 1; }
  echo "== cfg $c"; cut -c1-150 gpurun_out/ls_$c.log | grep -v amdgpu
done
