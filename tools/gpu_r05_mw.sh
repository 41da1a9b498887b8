#!/bin/bash
# Round-5 wide Miller loop (k_miller_wide) changes: its bit-exactness tests (every small-batch path, the
# RLC finish), the latency probe at 1 / 256 / 1,024 credentials, the RLC single call.  First failure ends.
set -o pipefail
OUT=gpurun_out/${1:-r05mw}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests -k "single_element or wide_miller or small_batch or rlc" > $OUT/pytest_mw.log 2>&1 || { tail -30 $OUT/pytest_mw.log; exit 1; }
tail -1 $OUT/pytest_mw.log
timeout -k 10 300 python -u tools/latency_probe.py --ns 1,256,1024 > $OUT/latency.jsonl 2> $OUT/latency.err || { tail -20 $OUT/latency.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/latency.jsonl'):
    d = json.loads(l); print(d['mode'], d['n'], d['ok'], d['device_ms_median'], d['phase_ms'])"
timeout -k 10 400 python -X faulthandler bench.py --mode rlc --steps 10 --warmup 2 --no-cpu-baseline > $OUT/rlc.json 2> $OUT/rlc.err || { tail -5 $OUT/rlc.err; exit 1; }
python3 -c "import json; d=json.loads(open('$OUT/rlc.json').read().strip().splitlines()[-1]); print('rlc', d['value'], d['ms_per_step'], d.get('single_call_ms'))"
