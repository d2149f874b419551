#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_bvh.py -x -q > gpurun_out/pytest_bvh.log 2>&1; rc=$?; echo "bvh tests rc=$rc"; tail -30 gpurun_out/pytest_bvh.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_bvh.json 2> gpurun_out/bench_bvh.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_bvh.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline --exhaustive > gpurun_out/bench_exh.json 2>&1; rc=$?; echo "bench-exh rc=$rc"; cat gpurun_out/bench_exh.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "all gpu tests rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
