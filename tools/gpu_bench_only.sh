#!/bin/bash
# Bench lines of the committed build (config 2 with CPU baseline, config 3), after a PMC summary refresh.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-bench_only}
mkdir -p "$OUT"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 600 python bench.py --mode rlc --steps 5 --warmup 1 > "$OUT/bench_rlc.json" 2> "$OUT/bench_rlc.err"
