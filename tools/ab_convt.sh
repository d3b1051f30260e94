#!/bin/bash
# UNet ConvTranspose2d(2,2) forward (scatter epilogue) per forced linear tile config (one box)
set -e
out=gpurun_out/ab_convt
mkdir -p $out
for c in auto A B D E; do
  if [ $c = auto ]; then e="STF_AB=0"; else e="STF_IGEMM_CFG=$c"; fi
  env $e timeout -k 10 200 python3 tools/bench_layers.py 64 > $out/$c.txt 2>&1
  echo "== $c"; grep "^up\|TOTAL convT" $out/$c.txt
done
