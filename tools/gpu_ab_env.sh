#!/bin/bash
# A/B on one box: GPU parity tests on the default build, then the verify (and RLC) benches alternating
# the default selection and an environment override ($2, e.g. CC_FEXP=pl).
# Usage (repo root, GPU box): bash tools/gpu_ab_env.sh <tag> <VAR=value> [tests|bench|all] [rlc]
set -o pipefail
TAG=${1:-ab}
OVR=${2:-CC_FEXP=pl}
WHAT=${3:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
    local t=$1 log=$2
    shift 2
    echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
    run 900 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    for r in 1 2; do
        run 300 "$OUT/bench_verify_new_$r.json" python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
        run 300 "$OUT/bench_verify_old_$r.json" env "$OVR" python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
    done
    if [ "${4:-}" = rlc ]; then
        run 300 "$OUT/bench_rlc_new.json" python -u bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline
        run 300 "$OUT/bench_rlc_old.json" env "$OVR" python -u bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline
    fi
fi
