#!/bin/bash
# Run GPU steps in order; each line of the step file is "<timeout_s> <log name> <command...>".
# An ordinary failure (exit 1..3, e.g. a failing test) goes on to the next step; a time limit,
# abort, segfault or kill (124/134/137/139, or >128) ends the run: nothing more touches the GPU.
#   bash bench/gpu_steps.sh <outdir> <stepfile>
out=${1:?outdir}; steps=${2:?stepfile}
mkdir -p "$out"
export TMPDIR=/tmp
while IFS= read -r line; do
  [[ -z "$line" || "$line" == \#* ]] && continue
  t=${line%% *}; rest=${line#* }; name=${rest%% *}; cmd=${rest#* }
  echo "[gpu_steps] $(date +%T) start $name: $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $(date +%T) end $name rc=$rc"
  tail -n 3 "$out/$name.log"
  if [[ $rc -eq 124 || $rc -eq 134 || $rc -eq 137 || $rc -eq 139 || $rc -gt 128 ]]; then
    echo "[gpu_steps] stopping after $name (rc=$rc)"; exit $rc
  fi
done < "$steps"
