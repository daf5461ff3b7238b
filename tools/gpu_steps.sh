#!/bin/bash
# Run GPU steps in order, each under its own time limit; a step that merely fails
# (exit 1, e.g. a test assertion) does not stop the ones after it, but a time
# limit (124 / 137), an abort (134) or a crash (139) -- anything that may have
# left the GPU in a bad state -- ends the call there.
#   bash tools/gpu_steps.sh OUTDIR "SECONDS NAME COMMAND..." ...
out=$1
shift
mkdir -p "$out"
status=0
for step in "$@"; do
  read -r secs name cmd <<< "$step"
  echo "== $name ($secs s): $cmd" | tee -a "$out/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.txt" 2>&1
  rc=$?
  echo "== $name rc=$rc" | tee -a "$out/steps.log"
  tail -3 "$out/$name.txt" | tee -a "$out/steps.log"
  if [ $rc -ne 0 ]; then status=$rc; fi
  case $rc in
    0|1|2) ;;
    *) echo "== stopping after $name (rc $rc)" | tee -a "$out/steps.log"; exit $rc ;;
  esac
done
exit $status
