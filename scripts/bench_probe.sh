#!/usr/bin/env bash
# GPU box: the default bench line plus the raw amd-smi clock JSON its clock sampler parses.
set -u
mkdir -p gpurun_out
(amd-smi metric -g 0 --clock --json > gpurun_out/amdsmi_clock.json 2>&1 || true)
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; tail -c 3000 gpurun_out/bench_default.json; tail -5 gpurun_out/bench_default.err; exit $rc
