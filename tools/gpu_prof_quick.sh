#!/bin/bash
# Quick per-kernel counter look (dev tool): kernel trace + a few PMC passes of
# prof_frames.py. Usage: bash tools/gpu_prof_quick.sh TAG [prof_frames args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=${1:-q}; shift
OUT=gpurun_out/profq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 120 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python tools/prof_frames.py --frames 3 $ARGS > $OUT/$name.log 2>&1; rc=$?; echo "$name rc=$rc"; return $rc; }
ARGS="$*"
run kt --kernel-trace --stats && \
run p1 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM && \
run p2 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS TCC_HIT_sum TCC_MISS_sum
