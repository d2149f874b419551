#!/bin/bash
# Profile the bench workload on the GPU box: rocprofv3 kernel-trace stats, then
# PMC passes (one counter group per run, never combined with sys/runtime
# traces), summarised per kernel class and per frame by tools/pmc_summary.py.
# Usage: [BATCH=B] bash tools/profile.sh TAG [tools/prof_frames.py args]
#        BATCH (default 8): frames per render call, as bench.py renders them
#        SUMMARY_ARGS="--width 4096 --height 4096 --spheres 9996" for a non-C3 workload.
# Output: gpurun_out/prof_TAG/ (copy kernel_stats / pmc_summary into profiles/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=${1:-r02}; shift
BATCH=${BATCH:-8}
ARGS="--frames $((5 * BATCH)) --batch $BATCH $*"
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  name=$1; shift
  timeout -s KILL 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
    python tools/prof_frames.py $ARGS > "$OUT/$name.log" 2>&1
  rc=$?; echo "$name rc=$rc" | tee -a "$OUT/steps.log"; return $rc
}
run kt --kernel-trace --stats && \
run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE && \
run p2 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VMEM && \
run p3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_FMA_F32 && \
run p4 --pmc FETCH_SIZE && \
run p5 --pmc WRITE_SIZE && \
run p6 --pmc TCC_HIT_sum TCC_MISS_sum && \
python tools/pmc_summary.py "$OUT/pmc_summary.json" --dominant "${DOMINANT:-closest}" --batch "$BATCH" --traversal "${TRAVERSAL:-bvh}" \
  --build "$(python raytracer-challenge-rs_amd/rtamd/buildinfo.py)" \
  $SUMMARY_ARGS "$OUT"/p1 "$OUT"/p2 "$OUT"/p3 "$OUT"/p4 "$OUT"/p5 "$OUT"/p6 > /dev/null && \
  echo "summary ok" | tee -a "$OUT/steps.log"
