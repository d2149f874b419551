#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/tune1
export TMPDIR=/tmp
timeout -k 10 300 python tools/tune.py --waves 3,4,5,6 --rounds 4 > gpurun_out/tune1/tune.log 2>&1 && \
rocprofv3 -L > gpurun_out/tune1/counters.txt 2>&1 ; \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d gpurun_out/tune1/pmc1 -o p --output-format csv -- python tools/tune.py --waves 4 --rounds 1 > gpurun_out/tune1/pmc1.log 2>&1; echo "pmc1 rc=$?"
