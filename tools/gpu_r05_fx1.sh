#!/bin/bash
# Round-5 one-element fexp (k_fexp1) change: its bit-exactness tests first (n = 1 everywhere, RLC), then
# the whole -m gpu suite, the latency probe, and the verify / RLC / PoK bench lines.  First failure ends.
set -o pipefail
OUT=gpurun_out/${1:-r05x}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests -k "single_element or fexp or wide_miller or rlc_single or test_sign_verify_1" > $OUT/pytest_fx1.log 2>&1 || { tail -30 $OUT/pytest_fx1.log; exit 1; }
tail -1 $OUT/pytest_fx1.log
timeout -k 10 600 $T tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/latency_probe.py --ns 1,16,256,1024,1025,4096 > $OUT/latency.jsonl 2> $OUT/latency.err || { tail -20 $OUT/latency.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/latency.jsonl'):
    d = json.loads(l); print(d['mode'], d['n'], d['ok'], d['device_ms_median'], d['phase_ms'])"
run() {  # name, args
  timeout -k 10 400 python -X faulthandler bench.py $2 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config'].get('batches_in_flight'), (d.get('default_tables') or {}).get('value'), d.get('single_call_ms'))"
}
run rlc "--mode rlc --steps 10 --warmup 2 --no-cpu-baseline"
run verify "--steps 20 --warmup 3 --no-cpu-baseline"
