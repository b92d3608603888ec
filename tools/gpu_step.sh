# Run GPU steps in order under their own time limits; a step that ends in a plain test failure (rc 1) lets the next
# ones run, anything else (fault, abort, segfault, time limit) stops the call.  Usage (from the repo root, via gpurun):
#   bash tools/gpu_step.sh OUTDIR "SECONDS NAME COMMAND..." ["SECONDS NAME COMMAND..." ...]
# Each step's stdout+stderr goes to OUTDIR/NAME.log.
O=$1
shift
mkdir -p "$O"
for step in "$@"; do
  secs=${step%% *}
  rest=${step#* }
  name=${rest%% *}
  cmd=${rest#* }
  echo "[gpu_step] $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.log" 2>&1
  rc=$?
  echo "[gpu_step] $name rc=$rc"
  tail -3 "$O/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "[gpu_step] stopping after $name (rc $rc)"
    exit $rc
  fi
done
exit 0
