#!/bin/bash
# One gpurun call = a chain of GPU steps, each under its own time limit; the
# chain stops at the first failing step (no GPU step after a fault/timeout).
# Usage (on the box): bash tools/gpu_job.sh TAG STEP [STEP ...]
#   tests      pytest -m gpu (thread-timeout per test)
#   smoke      __graft_entry__.smoke()
#   bench      python bench.py (default args) > TAG_bench.json
#   benchq     bench.py without the CPU baseline / end-to-end (quick)
#   c5         bench.py --config c5 --steps 3 --warmup 1 (no CPU baseline)
#   shard      tools/shard_time.py --ns 1,2,4,8
#   shardb     the same with 8-frame batches (rt_render_frames_device)
#   tsel       pytest -m gpu of the files in $TESTS
#   trace      rocprofv3 --kernel-trace --stats of the timed bench regime
#   trace_c5   the same for C5
#   pmc        tools/profile.sh TAG (kernel trace + PMC passes of 5 serialized frames)
#   pmc_c5     the same for C5
#   quick      tools/quick_time.py (C3 and C5 frame times, two runs)
#   ppm        tools/ppm_probe.py (where rt_render_ppm's time goes)
#   multi      tools/multi_probe.py (rt_render_multi's per-device parts, projected N-device frame)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name (limit ${secs}s): $*" | tee -a "$OUT/steps.log"
  local t0=$(date +%s)
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/$name.log"
  return $rc
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1 ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench) step bench 600 python bench.py || exit 1; grep '^{' "$OUT/bench.log" > "$OUT/bench.json" ;;
    benchq) step benchq 400 python bench.py --no-cpu-baseline --no-end-to-end || exit 1; grep '^{' "$OUT/benchq.log" > "$OUT/benchq.json" ;;
    c5) step c5 600 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline --no-end-to-end || exit 1 ;;
    shard) step shard 600 python tools/shard_time.py --ns 1,2,4,8 --frames 100 --ranks || exit 1 ;;
    shardb) step shardb 600 python tools/shard_time.py --ns 1,2,4,8 --frames 160 --batch 8 --ranks || exit 1 ;;
    tsel) step tsel 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 240 --timeout-method thread -p no:cacheprovider || exit 1 ;;
    trace) step trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o trace --output-format csv -- \
             python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end || exit 1 ;;
    trace_c5) step trace_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace_c5" -o trace_c5 --output-format csv -- \
             python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end || exit 1 ;;
    pmc) step pmc 900 bash tools/profile.sh "$TAG" || exit 1 ;;
    pmc_c5) BATCH=1 SUMMARY_ARGS="--width 4096 --height 4096 --spheres 9996" step pmc_c5 900 bash tools/profile.sh "${TAG}_c5" --config c5 --width 4096 --height 4096 --spheres 9996 || exit 1 ;;
    quick) step quick 600 python tools/quick_time.py || exit 1 ;;
    ppm) step ppm 300 python tools/ppm_probe.py || exit 1 ;;
    multi) step multi 300 python tools/multi_probe.py || exit 1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "job $TAG done"
