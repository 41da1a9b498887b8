#!/bin/bash
# rocprofv3 kernel stats of the RLC bench (config 3 slice).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${1:-prof_rlc}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o rlc --output-format csv -- python3 "$R/bench.py" --mode rlc --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/bench_rlc.json" 2> "$OUT/prof.err"
