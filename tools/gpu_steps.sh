#!/bin/bash
# One GPU call of several steps, each under its own time limit; stops at the
# first failure (tools/gpu_steps.sh OUTDIR STEP...), STEP = "name:seconds:command".
out=$1; shift
mkdir -p "$out"
for step in "$@"; do
  name=${step%%:*}; rest=${step#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.txt" 2>&1
  rc=$?
  echo "== $name rc=$rc"
  tail -3 "$out/$name.txt"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
