#!/bin/bash
# Round-5 small-batch Miller path: the new GPU test first, then the whole -m gpu suite, then the latency
# probe on the shipped build (kWideMax = 512) and on a variant (libcoconut_hip_vW.so, kWideMax = 2048)
# around the crossover.  First failure ends the script.
set -o pipefail
OUT=gpurun_out/${1:-r05w}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "wide_miller or ragged" > $OUT/pytest_wide.log 2>&1 || { tail -30 $OUT/pytest_wide.log; exit 1; }
tail -1 $OUT/pytest_wide.log
timeout -k 10 600 $T tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
NS=1,16,256,512,513,1024,2048,4096
timeout -k 10 300 python -u tools/latency_probe.py --ns $NS > $OUT/latency_cur.jsonl 2> $OUT/latency_cur.err || { tail -20 $OUT/latency_cur.err; exit 1; }
COCONUT_HIP_LIB=$(pwd)/coconut-rust_amd/libcoconut_hip_vW.so timeout -k 10 300 python -u tools/latency_probe.py --ns 1024,2048,4096 --modes 0 > $OUT/latency_vW.jsonl 2> $OUT/latency_vW.err || { tail -20 $OUT/latency_vW.err; exit 1; }
python3 - <<PY
import json
for f in ("$OUT/latency_cur.jsonl", "$OUT/latency_vW.jsonl"):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1], d["mode"], d["n"], d["ok"], d["device_ms_median"], d["phase_ms"])
PY
