#!/bin/bash
# Round-end evidence on one GPU box: parity tests, smoke, bench (config 2, with CPU baseline),
# bench --mode rlc (config 3 per-GPU slice), rocprofv3 kernel-trace stats of the bench, PMC passes.
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${1:-final}
mkdir -p "$OUT"
echo "[final] pytest -m gpu"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
echo "[final] smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
echo "[final] bench"
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "[final] bench rlc"
timeout -k 10 600 python bench.py --mode rlc --steps 5 --warmup 1 > "$OUT/bench_rlc.json" 2> "$OUT/bench_rlc.err"
echo "[final] bench modes"
timeout -k 10 600 python bench.py --mode verify-g1 --steps 5 --warmup 1 > "$OUT/bench_verify_g1.json" 2> "$OUT/bench_verify_g1.err"
timeout -k 10 600 python bench.py --mode aggregate --steps 3 --warmup 1 > "$OUT/bench_aggregate.json" 2> "$OUT/bench_aggregate.err"
timeout -k 10 600 python bench.py --mode pok --steps 3 --warmup 1 > "$OUT/bench_pok.json" 2> "$OUT/bench_pok.err"
echo "[final] rocprofv3 stats"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o bench --output-format csv -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
cd "$R"
echo "[final] pmc"
PMC_OUT="$OUT/pmc" bash tools/pmc_round.sh > "$OUT/pmc.log" 2>&1
echo "[final] done"
