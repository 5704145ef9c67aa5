#!/usr/bin/env bash
# Runs on the GPU box (via gpurun): each GPU step under its own time limit; stops at the
# first step that faults / aborts / times out (rc 124, 134, 137, 139 or >128), continues
# past ordinary test failures (rc 1) so that the bench still reports.
#   scripts/gpu_session.sh "<step1>" "<step2>" ...
set -u
mkdir -p gpurun_out
i=0
for step in "$@"; do
  i=$((i + 1))
  echo "=== step $i: $step" | tee -a gpurun_out/session.log
  bash -c "$step"
  rc=$?
  echo "=== step $i rc=$rc" | tee -a gpurun_out/session.log
  if [ $rc -ge 124 ]; then
    echo "=== stopping: step $i ended with rc=$rc (fault/timeout)" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
