#!/bin/bash
# A/B an environment toggle on the kernel tests + per-layer timings:  VAR=NAME VALUES="0 1" bash tools/ab_env.sh
mkdir -p gpurun_out
for v in ${VALUES:-0 1}; do
  env $VAR=$v timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/tab_$v.log 2>&1 || { echo "tests failed $VAR=$v"; tail -20 gpurun_out/tab_$v.log; exit 1; }
  env $VAR=$v timeout -k 10 200 python tools/bench_layers.py 64 > gpurun_out/lab_$v.log 2>&1 || exit 1
  echo "== $VAR=$v: $(tail -1 gpurun_out/tab_$v.log)"; grep -E "^(enc1.3|enc2.3|enc3.3|dec2.0|dec1.0|dec1.3|TOTAL)" gpurun_out/lab_$v.log | cut -c1-125
done
