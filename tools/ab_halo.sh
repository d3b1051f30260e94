#!/bin/bash
# A/B the halo conv epilogue (LDS-staged 16-B stores vs direct 8-B fragment stores)
mkdir -p gpurun_out
for d in 0 1; do
  STF_HALO_DIRECT=$d timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -x -q -k "halo or forward_stats or concat" > gpurun_out/th_$d.log 2>&1 || { echo "tests failed direct=$d"; tail -20 gpurun_out/th_$d.log; exit 1; }
  STF_HALO_DIRECT=$d timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/lh_$d.log 2>&1 || exit 1
  echo "== direct $d: $(tail -1 gpurun_out/th_$d.log)"; grep -E "^(enc1.3|enc2.3|enc3.3|dec2.0|dec1.0|dec1.3|TOTAL)" gpurun_out/lh_$d.log | cut -c1-125
done
