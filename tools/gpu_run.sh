#!/bin/bash
# run one python dev script on the GPU box with a time limit
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 ${TL:-300} python "$@" 2>&1 | grep -v amdgpu.ids | tee gpurun_out/run.log
