#!/bin/bash
# Round-2 GPU session: parity tests, micro-benchmark, benches of every mode, rocprof kernel stats.
# Usage (from the repo root, on the GPU box): bash tools/gpu_r02.sh <tag> [tests|bench|quick|modes|prof|all]
set -o pipefail
TAG=${1:-r02}
WHAT=${2:-all}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <seconds> <logfile> <cmd...>: stop the session on any failure
    local t=$1 log=$2
    shift 2
    echo "== $(date +%T) $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$t" "$@" > "$log" 2>&1
    local rc=$?
    echo "   rc=$rc" | tee -a "$OUT/steps.log"
    if [ $rc -ne 0 ]; then tail -30 "$log"; exit $rc; fi
}
if [ "$WHAT" = tests ] || [ "$WHAT" = all ]; then
    run 900 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
fi
if [ "$WHAT" = bench ] || [ "$WHAT" = all ]; then
    run 120 "$OUT/ubench_int.jsonl" tools/ubench_int
    run 400 "$OUT/bench_verify.json" python -u bench.py --steps 10 --warmup 2
    run 300 "$OUT/bench_verify_g1.json" python -u bench.py --mode verify-g1 --steps 5 --warmup 1 --no-cpu-baseline
    run 300 "$OUT/bench_rlc.json" python -u bench.py --mode rlc --steps 5 --warmup 1
    run 400 "$OUT/bench_aggregate.json" python -u bench.py --mode aggregate --steps 3 --warmup 1
    run 400 "$OUT/bench_pok.json" python -u bench.py --mode pok --steps 3 --warmup 1
fi
if [ "$WHAT" = quick ]; then
    run 900 "$OUT/pytest_gpu.log" python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"}
    run 300 "$OUT/bench_verify.json" python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline
    run 300 "$OUT/bench_rlc.json" python -u bench.py --mode rlc --steps 5 --warmup 1 --no-cpu-baseline
fi
if [ "$WHAT" = modes ]; then
    run 400 "$OUT/bench_aggregate.json" python -u bench.py --mode aggregate --steps 3 --warmup 1
    run 400 "$OUT/bench_pok.json" python -u bench.py --mode pok --steps 3 --warmup 1
fi
if [ "$WHAT" = prof ] || [ "$WHAT" = all ]; then
    run 400 "$OUT/rocprof.log" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
        python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline
fi
echo done | tee -a "$OUT/steps.log"
