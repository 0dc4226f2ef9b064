#!/bin/bash
# Bench variants by environment (GPU box), one short bench per line of the
# spec file (NAME ENV=VAL... [-- bench args]); each run's JSON + log under
# gpurun_out/<tag>/NAME.{json,log}, and the step line echoed.
# usage: tools/sweep_env.sh <tag> <spec-file>
set -uo pipefail
TAG=$1; SPEC=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
while read -r NAME REST; do
  [ -z "$NAME" ] && continue
  case $NAME in \#*) continue ;; esac
  ENVS=(); ARGS=()
  seen=0
  for w in $REST; do
    if [ "$w" = "--" ]; then seen=1; continue; fi
    if [ $seen -eq 0 ]; then ENVS+=("$w"); else ARGS+=("$w"); fi
  done
  echo "[sweep] $NAME ${ENVS[*]} ${ARGS[*]} $(date +%T)"
  env "${ENVS[@]}" timeout -k 10 300 python -u bench.py --no-cpu --no-gather "${ARGS[@]}" \
      > "$OUT/$NAME.json" 2> "$OUT/$NAME.log" || { echo "[sweep] $NAME failed rc=$?"; exit 1; }
  grep "step cold" "$OUT/$NAME.log" | sed 's/^/    /'
done < "$SPEC"
