#!/bin/bash
# A/B the halo kernel's minimum image width (STF_HALO_MINW 32 vs 16): UNet and STF layer shapes
mkdir -p gpurun_out
for v in 32 16; do
  STF_HALO_MINW=$v timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "halo or forward" > gpurun_out/tmw_$v.log 2>&1 || { tail -20 gpurun_out/tmw_$v.log; exit 1; }
  STF_HALO_MINW=$v timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/lmw_$v.log 2>&1 || exit 1
  STF_HALO_MINW=$v timeout -k 10 200 python tools/bench_layers.py --stf > gpurun_out/smw_$v.log 2>&1 || exit 1
  echo "== MINW=$v: $(tail -1 gpurun_out/tmw_$v.log)"; grep -E "^(bott|l3 |l4 |TOTAL fwd|TOTAL dgrad)" gpurun_out/lmw_$v.log gpurun_out/smw_$v.log | cut -c1-140
done
