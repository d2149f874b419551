#!/bin/bash
# A/B of bench.py variants on one box, alternating (dev tool; DESIGN.md's
# "alternating ... on one box" figures). Each variant is one quoted argument
# string appended to `python bench.py --no-cpu-baseline --no-end-to-end`;
# every variant runs ROUNDS times (default 2), in turn, each under its own time
# limit, and the chain stops at the first failure.
# Usage (on the box): bash tools/ab_bench.sh TAG "--knob prim_lane=0" "--knob prim_lane=1"
#        ROUNDS=3 bash tools/ab_bench.sh TAG "--batch 8 --inflight 4" "--batch 16 --inflight 3"
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p "$OUT"
for i in $(seq 1 "${ROUNDS:-2}"); do
  v=0
  for args in "$@"; do
    v=$((v + 1))
    log="$OUT/v${v}_$i.log"
    # shellcheck disable=SC2086
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-end-to-end $args > "$log" 2>&1 || { echo "variant $v failed: $args"; exit 1; }
    echo "$(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"closest": {"ms_per_frame": [0-9.]*\|"combine": {"ms_per_frame": [0-9.]*\|"ok": [a-z]*' "$log" | tr '\n' ' ') <- $args"
  done
done
