set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/abpl
for i in 1 2; do
  timeout -k 10 180 python bench.py --no-cpu-baseline --no-end-to-end --no-distinct --no-cold > gpurun_out/abpl/base_$i.log 2>&1 || exit 1
  timeout -k 10 180 python bench.py --no-cpu-baseline --no-end-to-end --no-distinct --no-cold --knob prim_lane=1 > gpurun_out/abpl/pl_$i.log 2>&1 || exit 1
done
echo ok
