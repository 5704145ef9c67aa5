#!/usr/bin/env bash
# One GPU-box session (run through gpurun): named steps, each under its own time limit, outputs in
# gpurun_out/<tag>/; stops at the first step that faults / aborts / times out (scripts/gpu_session.sh).
#   bash scripts/session.sh <tag> step [step ...]
# Steps (an optional VAR=value,VAR2=value prefix before '@' sets the environment of one step):
#   tests            the whole -m gpu suite                  -> <tag>/gpu_tests.txt
#   tests:<args>     pytest on a subset, e.g. tests:tests/test_gpu_parity.py,-k,paired
#   smoke            __graft_entry__.smoke()                  -> <tag>/smoke.txt
#   bench[:name]     the driver's bench command               -> <tag>/bench_<name>.json
#   profile          scripts/profile_round.sh <tag> bench (rocprofv3 trace + PMC passes of that command)
#   profile_headline the same, headline leg only
#   gloo2            two ranks sharing this GPU over gloo (the N > 1 path)  -> <tag>/bench_2ranks.json
#   sweep:<B,B,...>  bench lines at these batches (scripts/batch_sweep.sh)   -> <tag>/sweep_summary.txt
#   host:<B,B,...>   the host-pointer path next to the device path          -> <tag>/host_path.jsonl
#   tier1:<args>     tests/callers/_bin/tier1_rate <args>                    -> <tag>/tier1_rate.json
#   ab:<B>:<variants> scripts/ab_bench.sh at batch B                         -> <tag>/ab_<B>.txt
#   any other string is run as a shell command
# e.g. bash scripts/session.sh r05a tests smoke bench profile
set -u
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p "$O"
steps=()
for s in "$@"; do
  envp=""
  if [[ "$s" == *@* && "${s%%@*}" != *" "* ]]; then envp="${s%%@*}"; envp="${envp//,/ } "; s="${s#*@}"; fi
  case "$s" in
    tests) c="timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1" ;;
    tests:*) a="${s#tests:}"; c="timeout -k 10 600 python -u -m pytest ${a//,/ } -m gpu -x -v --timeout 300 --timeout-method thread >> $O/gpu_tests_subset.txt 2>&1" ;;
    smoke) c="timeout -k 10 300 python -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.txt 2>&1" ;;
    bench|bench:*) n="${s#bench}"; n="${n#:}"; n="${n:-default}"
      c="timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$n.json 2> $O/bench_$n.err" ;;
    profile) c="timeout -k 10 1150 bash scripts/profile_round.sh $TAG bench > $O/profile.txt 2>&1" ;;
    profile_headline) c="timeout -k 10 900 bash scripts/profile_round.sh $TAG headline > $O/profile.txt 2>&1" ;;
    gloo2) c="TFHE_AMD_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --host-batches none > $O/bench_2ranks.json 2> $O/bench_2ranks.err" ;;
    sweep:*) b="${s#sweep:}"; c="BATCHES='${b//,/ }' timeout -k 10 600 bash scripts/batch_sweep.sh $TAG/sweep > /dev/null 2>&1" ;;
    host:*) b="${s#host:}"; c="timeout -k 10 300 python scripts/host_path_rate.py ${b//,/ } >> $O/host_path.jsonl 2>&1" ;;
    tier1:*) a="${s#tier1:}"; c="timeout -k 10 300 tests/callers/_bin/tier1_rate ${a//,/ } >> $O/tier1_rate.json 2>&1" ;;
    ab:*) r="${s#ab:}"; b="${r%%:*}"; v="${r#*:}"
      c="AB_BATCH=$b AB_STEPS=20 AB_WARMUP=10 AB_REPS=2 timeout -k 10 600 bash scripts/ab_bench.sh ${v//,/ } > $O/ab_$b.txt 2>&1" ;;
    *) c="$s" ;;
  esac
  steps+=("$envp$c")
done
if [ -n "${DRY:-}" ]; then printf '%s\n' "${steps[@]}"; exit 0; fi
bash scripts/gpu_session.sh "${steps[@]}"
exit $?
