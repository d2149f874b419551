#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/tune4
#timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/tune4/pytest.log 2>&1; echo "pytest rc=$?"
timeout -k 10 300 python tools/tune.py --knob wf_waves --waves 8,4 --rounds 5 > gpurun_out/tune4/tune.log 2>&1; echo "tune rc=$?"
