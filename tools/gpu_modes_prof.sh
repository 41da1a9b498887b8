#!/bin/bash
# Per-mode evidence for configs 3/4/5 (and SigG1 config 2): rocprofv3 kernel-trace stats of a short
# bench run, then the PMC passes of tools/pmc_round.sh, one directory per mode.
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
TAG=${1:-modes}
shift || true
MODES=${*:-verify verify-g1 verify-pervk rlc aggregate pok}
export TMPDIR=/tmp
for m in $MODES; do
  OUT=$R/gpurun_out/$TAG/$m
  mkdir -p "$OUT"
  echo "[modes] $m: rocprofv3 stats"
  # --inflight 1: one batch at a time, so each launch's duration is the kernel's own (two batches in
  # flight co-run and stretch every launch) and agrees with the bench line's per-kernel table
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 "$R/bench.py" --mode $m --steps 20 --warmup 2 --no-cpu-baseline --no-pcie --no-sigg1 --inflight 1 > "$OUT/prof_bench.json" 2> "$OUT/prof.err")
  echo "[modes] $m: pmc"
  PMC_OUT="$OUT/pmc" BENCH_ARGS="--mode $m" bash tools/pmc_round.sh > "$OUT/pmc.log" 2>&1
  python3 tools/pmc_summary.py "$OUT/pmc" "$OUT/pmc_summary.json" > "$OUT/pmc_summary.log" 2>&1
done
echo "[modes] done"
