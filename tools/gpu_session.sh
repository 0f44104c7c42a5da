#!/bin/bash
# Runs GPU steps in order; a step that fails with a test failure (rc 1) lets the session go on,
# anything that looks like a crash / fault / timeout (rc >= 2 other than 5 = no tests) stops it.
# usage: tools/gpu_session.sh "<name>:<timeout>:<command>" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (timeout ${tmo}s) $cmd" | tee -a gpurun_out/session.log
  start=$(date +%s)
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc after $(( $(date +%s) - start ))s" | tee -a gpurun_out/session.log
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then
    echo "=== stopping session: step $name ended with rc=$rc" | tee -a gpurun_out/session.log
    exit $rc
  fi
done
exit 0
