#!/bin/bash
# Sweep the forced DMA tile (STF_IGEMM_CFG) over the ConvT 2x2 forward / dgrad shapes.
set -e
cd "$(dirname "$0")/.."
for c in ${CFGS:-auto A B C D E}; do
  if [ "$c" = auto ]; then
    timeout -k 10 120 python tools/convt_cfg.py "${1:-64}"
  else
    STF_IGEMM_CFG=$c timeout -k 10 120 python tools/convt_cfg.py "${1:-64}"
  fi
done
