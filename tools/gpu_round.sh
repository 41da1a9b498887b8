#!/bin/bash
# One GPU-box pass: parity tests -> smoke -> bench -> rocprofv3 kernel trace of the bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-5}
echo "[round] pytest -m gpu"; timeout -k 10 900 python -m pytest tests -m gpu -x -q --timeout=600 -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
echo "[round] smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "[round] bench"; timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 2 > "$OUT/bench.log" 2>&1
echo "[round] rocprofv3"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1
echo "[round] done"
