#!/bin/bash
# Round profile collection (GPU box, repo root), all on ONE box so the numbers agree:
#   1. the bench lines (python bench.py [--model stf], default steps)
#   2. rocprofv3 --kernel-trace --stats of the same workloads (per-kernel averages that
#      the bench line's roofline avg_launch_us is checked against; without the dice / CPU
#      legs, whose training steps would mix other shapes into the statistics)
#   3. the two PMC passes (HBM traffic, tools/pmc_passes.sh) per model -> pmc_traffic_*.json
#   4. the PK-map fit bench (tools/bench_pk.py) under rocprofv3, the eval-metric micro-bench
# Outputs (summaries only) under gpurun_out/prof_<tag>; copy into profiles/<tag>.
set -e
tag=${1:-r04}
root=$GRAFT_REPO_ROOT
out=$root/gpurun_out/prof_$tag
mkdir -p $out
if [ -z "$ONLY_PMC" ]; then
timeout -k 10 600 python3 bench.py > $out/bench_unet256_b64.json 2> $out/bench_unet.err
timeout -k 10 600 python3 bench.py --model stf > $out/bench_stf256_t8_b16.json 2> $out/bench_stf.err
timeout -k 10 600 python3 bench.py --config 4 --steps 20 --warmup 5 > $out/bench_cfg4_stf256_t16_b16.json 2> $out/bench_cfg4.err
timeout -k 10 600 python3 bench.py --config 5 --steps 10 --warmup 3 > $out/bench_cfg5_stf512_t32pk_b4_fp16.json 2> $out/bench_cfg5.err
timeout -k 10 600 python3 bench.py --dtype fp16 --no-cpu-baseline > $out/bench_unet256_b64_fp16.json 2> $out/bench_unet16.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/unet -o run -- \
  python3 $root/bench.py --no-dice --no-cpu-baseline > $out/unet_rocprof_bench.json 2> $out/unet.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/stf -o run -- \
  python3 $root/bench.py --model stf --no-dice --no-cpu-baseline > $out/stf_rocprof_bench.json 2> $out/stf.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/cfg5 -o run -- \
  python3 $root/bench.py --config 5 --steps 10 --warmup 3 --no-dice --no-cpu-baseline > $out/cfg5_rocprof_bench.json 2> $out/cfg5.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/pk -o run -- \
  python3 $root/tools/bench_pk.py > $out/bench_pk.json 2> $out/pk.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/aug -o run -- \
  python3 $root/tools/bench_aug.py > $out/aug_rocprof_bench.json 2> $out/aug.log
cd $root
timeout -k 10 200 python3 tools/bench_eval.py > $out/bench_eval.txt 2>&1
timeout -k 10 200 python3 tools/bench_aug.py > $out/bench_aug.json 2> $out/bench_aug.err
cp $out/unet/run_kernel_stats.csv $out/unet256_b64_kernel_stats.csv
cp $out/stf/run_kernel_stats.csv $out/stf256_t8_b16_kernel_stats.csv
cp $out/cfg5/run_kernel_stats.csv $out/cfg5_stf512_t32pk_b4_fp16_kernel_stats.csv
cp $out/pk/run_kernel_stats.csv $out/pk_fit256_kernel_stats.csv
cp $out/aug/run_kernel_stats.csv $out/aug_b16_kernel_stats.csv
rm -rf $out/unet $out/stf $out/cfg5 $out/pk $out/aug
fi
if [ -z "$SKIP_PMC" ]; then
bash tools/pmc_passes.sh gpurun_out/prof_$tag/pmc_unet --steps 3 --warmup 1
bash tools/pmc_passes.sh gpurun_out/prof_$tag/pmc_stf --model stf --steps 3 --warmup 1
bash tools/pmc_mfma.sh gpurun_out/prof_$tag/mfma_unet --steps 3 --warmup 1
bash tools/pmc_mfma.sh gpurun_out/prof_$tag/mfma_stf --model stf --steps 3 --warmup 1
python3 tools/pmc_mfma_summary.py gpurun_out/prof_$tag/mfma_unet --unet-layers \
  --workload "cfg2 UNet(in=8,base_c=64) 256x256 train step" --command "bash tools/pmc_mfma.sh OUT --steps 3 --warmup 1" \
  --json $out/pmc_mfma_unet256_b64.json > $out/pmc_mfma_unet256_b64_summary.txt
python3 tools/pmc_mfma_summary.py gpurun_out/prof_$tag/mfma_stf \
  --workload "cfg3 STFLSTMUNet(T=8) 256x256 train step" --command "bash tools/pmc_mfma.sh OUT --model stf --steps 3 --warmup 1" \
  --json $out/pmc_mfma_stf256_t8_b16.json > $out/pmc_mfma_stf256_t8_b16_summary.txt
python3 tools/pmc_summary.py gpurun_out/prof_$tag/pmc_unet --batch 64 \
  --workload "cfg2 UNet(in=8,base_c=64) 256x256 train step" \
  --command "bash tools/pmc_passes.sh OUT --steps 3 --warmup 1" --json $out/pmc_traffic_unet256_b64.json > $out/pmc_unet256_b64_summary.txt
python3 tools/pmc_summary.py gpurun_out/prof_$tag/pmc_stf --batch 16 \
  --workload "cfg3 STFLSTMUNet(T=8) 256x256 train step" \
  --command "bash tools/pmc_passes.sh OUT --model stf --steps 3 --warmup 1" --json $out/pmc_traffic_stf256_t8_b16.json > $out/pmc_stf256_t8_b16_summary.txt
fi
rm -rf $out/pmc_unet $out/pmc_stf $out/mfma_unet $out/mfma_stf
ls $out
