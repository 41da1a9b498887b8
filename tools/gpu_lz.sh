#!/bin/bash
# Lazy-field A/B session on one box: GPU parity tests on the default build with every Miller selection
# (CC_MILLER = lz | pl | default), then the verify and RLC benches under each selection.
# Usage (repo root, GPU box): bash tools/gpu_lz.sh <tag> [tests|bench|all]
set -o pipefail
TAG=${1:-lz}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
    local t=$1 log=$2
    shift 2
    echo "== $(date +%T) CC_MILLER=${CC_MILLER:-} $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
    run 900 "$OUT/pytest_gpu_lz.log" python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    for m in lz pl lz pl; do
        CC_MILLER=$m run 300 "$OUT/bench_verify_$m.json" python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
        cp "$OUT/bench_verify_$m.json" "$OUT/bench_verify_${m}_$(date +%s).json"
    done
    CC_MILLER=lz run 300 "$OUT/bench_rlc_lz.json" python -u bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline
    CC_MILLER=pl run 300 "$OUT/bench_rlc_pl.json" python -u bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline
fi
