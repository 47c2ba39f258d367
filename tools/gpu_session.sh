#!/bin/bash
# Runs a list of GPU steps (one per line in $1), each under its own timeout.
# Test failures (exit 1) continue; faults / aborts / timeouts (124,134,137,139, >128) stop the session.
# Usage: bash tools/gpu_session.sh steps.txt   (lines: "<timeout_s> <logname> <command...>")
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
while IFS= read -r line || [ -n "$line" ]; do
  [ -z "$line" ] && continue
  case "$line" in \#*) continue;; esac
  t=$(echo "$line" | awk '{print $1}')
  name=$(echo "$line" | awk '{print $2}')
  cmd=$(echo "$line" | cut -d' ' -f3-)
  echo "=== [$name] (timeout ${t}s) $cmd"
  start=$(date +%s)
  timeout -k 10 "$t" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  end=$(date +%s)
  echo "=== [$name] rc=$rc in $((end-start))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then
    echo "=== stopping: step $name ended with rc=$rc (fault/timeout/abort)"
    exit $rc
  fi
done < "$1"
