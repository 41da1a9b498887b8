#!/bin/bash
# A/B on one GPU box: parity tests (pair-lane default), then bench in both lane layouts.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
echo "[ab] pytest -m gpu (pair-lane)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout=300 -p no:cacheprovider > "$OUT/pytest_gpu_pl.log" 2>&1
echo "[ab] bench pair-lane"
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench_pl.log" 2>&1
echo "[ab] done"
