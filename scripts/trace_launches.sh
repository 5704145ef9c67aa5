set -u
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for B in 1024 4096; do
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tr_$B -o run -- python3 $R/bench.py --steps 12 --warmup 2 --batch $B --no-cpu-baseline --no-clock --no-ceiling --extra-batches none --strong-batch 0 > $R/gpurun_out/tr_$B.log 2>&1 || exit 3
done
