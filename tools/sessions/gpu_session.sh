#!/bin/bash
# Runs GPU steps in order; each under its own time limit.  Test failures (exit 1) do not stop
# the session; a crash, abort, fault or timeout does (no further GPU work after it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/session.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
