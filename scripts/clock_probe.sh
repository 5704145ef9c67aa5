#!/usr/bin/env bash
# Samples the GPU's shader clock / power while a long bench runs (GPU box, diagnostics only).
#   bash scripts/clock_probe.sh <batch> <steps>
set -u
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps ${2:-400} --warmup 2 --batch ${1:-1024} --no-cpu-baseline > gpurun_out/clk_bench_$1.json 2>&1 &
pid=$!
for k in $(seq 1 12); do
  sleep 1
  (amd-smi metric -g 0 --clock --power 2>&1 || rocm-smi --showclocks --showpower 2>&1) | grep -iE "gfx|sclk|power|socket|clk" | head -12 >> gpurun_out/clk_$1.log
  echo "---" >> gpurun_out/clk_$1.log
  kill -0 $pid 2>/dev/null || break
done
wait $pid
