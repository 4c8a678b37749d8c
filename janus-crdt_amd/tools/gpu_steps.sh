#!/bin/bash
# gpu_steps.sh LOG SECONDS CMD... — one GPU step of a gpurun call: runs CMD under its own time limit with
# output to gpurun_out/LOG, and stops the call (exit != 0) on anything worse than a failed test (pytest
# exit 1): a fault, an abort, a signal or a time limit.  Chain steps with &&.
log="gpurun_out/$1"; secs="$2"; shift 2
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "rc=$rc" >> "$log"
echo "[$log] rc=$rc"
[ "$rc" -le 1 ] || exit "$rc"
