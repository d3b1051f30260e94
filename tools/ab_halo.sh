#!/bin/bash
# A/B the halo conv variants (STF_HALO_VARIANT: 0 = 16x32 8-wave 2-stage, 1 = 8x32 4-wave single stage x2 WG/CU)
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1}; do
  STF_HALO_VARIANT=$v timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -x -q -k "halo or forward_stats or concat" > gpurun_out/th_$v.log 2>&1 || { echo "tests failed variant=$v"; tail -20 gpurun_out/th_$v.log; exit 1; }
  STF_HALO_VARIANT=$v timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/lh_$v.log 2>&1 || exit 1
  echo "== variant $v: $(tail -1 gpurun_out/th_$v.log)"; grep -E "^(enc1.3|enc2.3|enc3.3|enc4.3|dec2.0|dec1.0|dec1.3|TOTAL)" gpurun_out/lh_$v.log | cut -c1-125
done
