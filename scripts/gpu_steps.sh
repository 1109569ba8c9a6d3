#!/bin/bash
# GPU box: run steps one after another, each under its own time limit, and stop at the first step that
# timed out, aborted or crashed (124, 137, 134, 139, or any status above 128): after such a step nothing
# more touches the GPU in this call. An ordinary failure (a failed test: status 1) does not stop the chain.
#   scripts/gpu_steps.sh <seconds> '<command>' [<seconds> '<command>' ...]
rc_all=0
while [ $# -ge 2 ]; do
  t=$1; cmd=$2; shift 2
  echo "[gpu_steps] $(date +%T) start: $cmd"
  timeout -k 10 "$t" bash -c "$cmd"
  rc=$?
  echo "[gpu_steps] $(date +%T) exit $rc: $cmd"
  if [ $rc -ne 0 ]; then rc_all=$rc; fi
  if [ $rc -eq 124 ] || [ $rc -gt 128 ]; then
    echo "[gpu_steps] stopping after exit $rc"
    exit $rc
  fi
done
exit $rc_all
