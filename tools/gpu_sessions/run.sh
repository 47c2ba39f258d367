#!/bin/bash
# Runs a list of GPU steps (one per line in $1), each under its own timeout.
# Any nonzero exit stops the session (a pytest failure can be a GPU memory fault: nothing more runs on the GPU after it).
# Usage: bash tools/gpu_sessions/run.sh tools/gpu_sessions/<steps>.txt   (lines: "<timeout_s> <logname> <command...>")
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
  if [ $rc -ne 0 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done < "$1"
