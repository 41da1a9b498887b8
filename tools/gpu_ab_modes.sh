#!/bin/bash
# Same-box A/B of the previous library build (libcoconut_hip_prev.so) against the current one over several
# bench modes, after the GPU test suite (TESTS, default all of tests/ marked gpu).  Each GPU step has its
# own time limit; the first failure ends the script.  Usage: [MODES="verify rlc"] bash tools/gpu_ab_modes.sh <tag>
set -o pipefail
TAG=${1:-abm}
OUT=gpurun_out/$TAG
MODES=${MODES:-verify aggregate rlc pok}
TESTS=${TESTS:-tests}
mkdir -p "$OUT"
echo "[abm] tests $TESTS"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for m in $MODES; do
  for v in prev cur; do
    lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
    [ $v = prev ] && lib=$(pwd)/coconut-rust_amd/libcoconut_hip_prev.so
    [ -f "$lib" ] || continue
    echo "[abm] bench $m $v"
    COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --mode $m --steps 5 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/${m}_$v.json" 2> "$OUT/${m}_$v.err" || exit 1
  done
done
echo "[abm] done"
