#!/bin/bash
# Round evidence on one GPU box, part 1: parity tests, smoke, the bench line of every mode (config 2
# with its CPU baseline, SigG1, per-credential verkeys, RLC, aggregate, PoK).  Part 2 (rocprofv3 kernel stats and PMC passes per
# mode) is tools/gpu_modes_prof.sh.  Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${1:-final}
mkdir -p "$OUT"
echo "[final] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
tail -1 "$OUT/pytest_gpu.log"
echo "[final] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "[final] bench"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
for m in verify-g1 verify-pervk verify-pervk-g1 rlc aggregate pok aggregate-g1 pok-g1; do
  echo "[final] bench $m"
  timeout -k 10 600 python bench.py --mode $m --steps 5 --warmup 1 > "$OUT/bench_$m.json" 2> "$OUT/bench_$m.err"
done
echo "[final] done"
