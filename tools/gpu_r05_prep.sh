#!/bin/bash
# Round-5 wide prep: the small-batch parity tests, the whole -m gpu suite, the latency probe, then the
# remaining modes' rocprofv3 stats + PMC passes (tools/gpu_modes_prof.sh).  First failure ends.
set -o pipefail
OUT=gpurun_out/${1:-r05p}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "wide_miller or ragged or concurrent or identity or infinity" > $OUT/pytest_wide.log 2>&1 || { tail -30 $OUT/pytest_wide.log; exit 1; }
tail -1 $OUT/pytest_wide.log
timeout -k 10 600 $T tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/latency_probe.py --ns 1,16,256,1024,2048,2049 > $OUT/latency.jsonl 2> $OUT/latency.err || { tail -20 $OUT/latency.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/latency.jsonl'):
    d = json.loads(l); print(d['mode'], d['n'], d['ok'], d['device_ms_median'], d['phase_ms'])"
bash tools/gpu_modes_prof.sh ${2:-r05modes2} aggregate pok verify-pervk-g1 aggregate-g1 pok-g1
