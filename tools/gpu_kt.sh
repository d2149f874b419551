#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=${1:-kt}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/kt -o kt --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/kt.log 2>&1; echo "kt rc=$?"
