#!/bin/bash
# Round-end measurement of the last build in one gpurun call (dev tool): GPU tests + smoke, the PMC passes of C3
# and C5 (their summaries placed in profiles/ under TAG so that bench.py finds this build's traffic), then the
# C3 and C5 bench lines and their kernel traces. Stops at the first failing step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
TAG=${1:-r06n}
bash tools/gpu_job.sh "$TAG" tests smoke pmc pmc_c5 || exit 1
cp "gpurun_out/prof_$TAG/pmc_summary.json" "profiles/${TAG}_pmc_summary.json" || exit 1
cp "gpurun_out/prof_${TAG}_c5/pmc_summary.json" "profiles/${TAG}_pmc_summary_c5.json" || exit 1
mkdir -p "gpurun_out/$TAG/profiles" && cp "profiles/${TAG}_pmc_summary.json" "profiles/${TAG}_pmc_summary_c5.json" "gpurun_out/$TAG/profiles/"
bash tools/gpu_job.sh "$TAG" bench c5 trace trace_c5
