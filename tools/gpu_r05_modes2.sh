#!/bin/bash
# Round-5 bench lines after the in-flight default: each verify mode at its default (2 batches in flight)
# and at --inflight 1, plus the RLC line (pipelined default-table leg).  First failure ends the script.
set -o pipefail
OUT=gpurun_out/${1:-r05d}
mkdir -p $OUT
run() {  # name, args
  timeout -k 10 400 python -X faulthandler bench.py $2 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config'].get('batches_in_flight'), (d.get('default_tables') or {}).get('value'), d.get('single_call_ms'))"
}
timeout -k 10 300 python -u -X faulthandler -m pytest tests/test_gpu_parity.py tests/test_gpu_rlc.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "concurrent or slots" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
run verify "--steps 20 --warmup 5"
run verify_if1 "--steps 20 --warmup 5 --inflight 1"
run verify_b "--steps 20 --warmup 5"
run verify-g1 "--mode verify-g1 --steps 20 --warmup 3 --no-cpu-baseline"
run verify-pervk "--mode verify-pervk --steps 10 --warmup 2 --no-cpu-baseline"
run verify-pervk_if1 "--mode verify-pervk --steps 10 --warmup 2 --no-cpu-baseline --inflight 1"
run verify-pervk-g1 "--mode verify-pervk-g1 --steps 10 --warmup 2 --no-cpu-baseline"
run rlc "--mode rlc --steps 10 --warmup 2 --no-cpu-baseline --rlc-inflight 1"
run rlc_if2 "--mode rlc --steps 10 --warmup 2 --no-cpu-baseline --rlc-inflight 2"
run rlc_if3 "--mode rlc --steps 10 --warmup 2 --no-cpu-baseline --rlc-inflight 3"
