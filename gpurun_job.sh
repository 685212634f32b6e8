#!/bin/bash
# helper for gpurun sessions: run steps in order, stop at the first crash/timeout
# (exit codes other than 0/1), never retry a GPU step.
set -u
mkdir -p gpurun_out
step() {  # step <name> <timeout_s> <cmd...>
    local name=$1 to=$2; shift 2
    echo "=== $name" >&2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc" >&2
    tail -5 "gpurun_out/$name.log" >&2
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)" >&2; exit $rc; fi
    return 0
}
