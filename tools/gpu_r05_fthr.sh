#!/bin/bash
# Round-5 fexp threshold (kFexpWideMax 1,024 -> 2,048, preps at kPrepWideMax 1,024): the small-batch
# path tests, the latency probe across the thresholds, the PoK / per-verkey lines.  First failure ends.
set -o pipefail
OUT=gpurun_out/${1:-r05ft}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 500 $T tests -k "small_batch or single_element or wide_miller or degenerate or identity_verkey or rlc" > $OUT/pytest_thr.log 2>&1 || { tail -30 $OUT/pytest_thr.log; exit 1; }
tail -1 $OUT/pytest_thr.log
timeout -k 10 300 python -u tools/latency_probe.py --ns 1,1024,1025,2048,2049,3072,4096,4097 > $OUT/latency.jsonl 2> $OUT/latency.err || { tail -20 $OUT/latency.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/latency.jsonl'):
    d = json.loads(l); print(d['mode'], d['n'], d['ok'], d['device_ms_median'], d['phase_ms'])"
