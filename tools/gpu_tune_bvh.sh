#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_bvh.py "$1" "$2" 2>&1 | tee gpurun_out/tune_bvh.log
