#!/bin/bash
# A/B the implicit-GEMM tile configurations: kernel parity + per-layer timing per config.
set -e
mkdir -p gpurun_out
for c in ${CFGS:-0 A B C D}; do  # 0 = auto, L = auto without the halo kernel, H = halo wherever eligible
  STF_IGEMM_CFG=$c timeout -k 10 200 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/t_$c.log 2>&1 || { echo "tests failed cfg $c"; tail -30 gpurun_out/t_$c.log; exit 1; }
  STF_IGEMM_CFG=$c timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/layers_$c.log 2>&1
  echo "== cfg $c: $(tail -1 gpurun_out/t_$c.log)"
  grep TOTAL gpurun_out/layers_$c.log
done
