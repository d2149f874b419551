#!/bin/bash
# Time library variants on one box, alternating (dev tool, on the GPU box):
#   ROUNDS=2 bash tools/archive/exp_time.sh TAG [ARGS="--config c3"] base NAME[:k=v,k=v] [...]
# `base` is the default build (lib/); NAME is lib_exp_NAME (tools/archive/exp_build.sh);
# ":k=v,..." adds tuning knobs (quick_time.py --knob) to that variant.
# Each run is tools/quick_time.py under its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=$1; shift
OUT=gpurun_out/exp_$TAG
mkdir -p "$OUT"
PKG=raytracer-challenge-rs_amd
for i in $(seq 1 "${ROUNDS:-2}"); do
  for v in "$@"; do
    lib=${v%%:*}
    knobs=""
    if [ "$lib" != "$v" ]; then for kv in $(echo "${v#*:}" | tr ',' ' '); do knobs="$knobs --knob $kv"; done; fi
    if [ "$lib" = base ]; then lp=""; else lp="$PWD/$PKG/lib_exp_$lib"; fi
    log="$OUT/$(echo "$v" | tr ':,=' '___')_$i.log"
    # shellcheck disable=SC2086
    LD_LIBRARY_PATH="$lp${LD_LIBRARY_PATH:+:$LD_LIBRARY_PATH}" timeout -k 10 240 \
      python tools/quick_time.py --tag "$v" $knobs ${ARGS:-} > "$log" 2>&1 || { echo "variant $v failed"; tail -5 "$log"; exit 1; }
    grep '^{' "$log" | tail -1
  done
done
