# C5 / C3 timing probes of the fast path (dev): one JSON line per variant.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/exp.jsonl
: > $OUT
Q="timeout -k 10 240 python tools/quick_time.py"
$Q --config c3 --frames 30 --tag c3 >> $OUT 2>/dev/null &&
$Q --config c5 --frames 3 --tag c5 >> $OUT 2>/dev/null
