set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out/lat
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/lat/tr -o tr -- python tools/prof_frames.py --frames 30 > gpurun_out/lat/run.log 2>&1
