#!/bin/bash
# Round-5 evidence on one GPU box: the whole -m gpu suite, smoke, the bench line of every mode (with the
# default-table legs and the RLC single-call latency), the Fp2-product micro-benchmark.  Each GPU step has
# its own time limit; the first failure ends the script.  Usage: bash tools/gpu_r05_evidence.sh <tag> [modes]
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ev}
MODES=${2:-"verify verify-g1 verify-pervk verify-pervk-g1 rlc aggregate aggregate-g1 pok pok-g1"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  echo "[ev] pytest -m gpu"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1
  tail -1 "$OUT/pytest_gpu.log"
  echo "[ev] smoke"
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
fi
for m in $MODES; do
  echo "[ev] bench $m"
  steps=20; [ "$m" = verify ] || steps=10
  timeout -k 10 600 python bench.py --mode $m --steps $steps --warmup 2 > "$OUT/bench_$m.json" 2> "$OUT/bench_$m.err"
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_$m.json').read().strip().splitlines()[-1]); print('$m', d['value'], d.get('default_tables',{}).get('value'), d.get('single_call_ms'))"
done
for k in ${INFLIGHT:-2 3}; do
  echo "[ev] bench verify --inflight $k"
  timeout -k 10 600 python bench.py --mode verify --steps 20 --warmup 2 --inflight $k --no-cpu-baseline > "$OUT/bench_verify_inflight$k.json" 2> "$OUT/bench_verify_inflight$k.err"
  python3 -c "import json; d=json.loads(open('$OUT/bench_verify_inflight$k.json').read().strip().splitlines()[-1]); print('inflight $k', d['value'], d['ms_per_step'])"
done
if [ -x tools/ubench_f2kara ]; then
  echo "[ev] ubench_f2kara"
  timeout -k 10 120 ./tools/ubench_f2kara > "$OUT/ubench_f2kara.jsonl" 2>&1
  cat "$OUT/ubench_f2kara.jsonl"
fi
echo "[ev] done"
