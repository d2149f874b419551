#!/bin/bash
# GPU round trip: all GPU tests, then the headline bench (no CPU baseline) + per-class times.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "gpu tests rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --no-cpu-baseline $* > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; }
python -c "
import json; d=json.load(open('gpurun_out/bench.json')); r=d['roofline']
print('value', d['value'], d['unit'], 'ms/step', d['ms_per_step'], 'frac', r['frac'], r.get('traversal'))
for k,v in r['kernels'].items(): print('  ', k, v)
"
