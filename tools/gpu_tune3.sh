#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/tune3
timeout -k 10 300 python tools/tune.py --waves 0,20 --rounds 5 > gpurun_out/tune3/tune.log 2>&1; echo "tune rc=$?"
