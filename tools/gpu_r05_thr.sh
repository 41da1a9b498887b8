#!/bin/bash
# Round-5 small-batch thresholds: the wide-path parity test, the latency probe around kWideMax = 2,048 on
# the shipped build and a kWideMax = 4,096 variant (libcoconut_hip_vW4.so).  First failure ends.
set -o pipefail
OUT=gpurun_out/${1:-r05t}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "wide_miller or ragged or concurrent" > $OUT/pytest_wide.log 2>&1 || { tail -30 $OUT/pytest_wide.log; exit 1; }
tail -1 $OUT/pytest_wide.log
timeout -k 10 300 python -u tools/latency_probe.py --ns 1,1024,1025,1536,2048,2049,4096 > $OUT/latency_cur.jsonl 2> $OUT/latency_cur.err || { tail -20 $OUT/latency_cur.err; exit 1; }
COCONUT_HIP_LIB=$(pwd)/coconut-rust_amd/libcoconut_hip_vW4.so timeout -k 10 300 python -u tools/latency_probe.py --ns 3072,4096 --modes 0 > $OUT/latency_vW4.jsonl 2> $OUT/latency_vW4.err || { tail -20 $OUT/latency_vW4.err; exit 1; }
python3 - <<PY
import json
for f in ("$OUT/latency_cur.jsonl", "$OUT/latency_vW4.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1], d["mode"], d["n"], d["ok"], d["device_ms_median"], d["phase_ms"])
PY
