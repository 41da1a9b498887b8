#!/bin/bash
# Same-box A/B with alternation (prev, cur, prev, cur): box clocks drift within a call by a few per
# cent, so single runs of each build do not separate small differences.  GPU tests (TESTS, default
# tests/) first.  Usage: [MODE=rlc] [TESTS=...] [REPS=2] bash tools/gpu_ab_alt.sh <tag>
set -o pipefail
TAG=${1:-abalt}
OUT=gpurun_out/$TAG
MODE=${MODE:-rlc}
TESTS=${TESTS:-tests}
REPS=${REPS:-2}
mkdir -p "$OUT"
[ -f coconut-rust_amd/libcoconut_hip_prev.so ] || { echo "[abalt] no coconut-rust_amd/libcoconut_hip_prev.so (build the previous version there first)"; exit 2; }
echo "[abalt] tests $TESTS"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for r in $(seq 1 "$REPS"); do
  for v in prev cur; do
    lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
    [ $v = prev ] && lib=$(pwd)/coconut-rust_amd/libcoconut_hip_prev.so
    echo "[abalt] $MODE $v $r"
    COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --mode "$MODE" --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/${MODE}_${v}_$r.json" 2> "$OUT/${MODE}_${v}_$r.err" || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d.get('phase_ms'))" "$OUT/${MODE}_${v}_$r.json"
  done
done
echo "[abalt] done"
