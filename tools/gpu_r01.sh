#!/bin/bash
# GPU session script: tests, bench, kernel-trace profile. Each GPU step has its own limit; stop at first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo "pytest rc=$?" | tee -a gpurun_out/steps.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc" | tee -a gpurun_out/steps.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o kt --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1; echo "rocprof rc=$?" | tee -a gpurun_out/steps.log
