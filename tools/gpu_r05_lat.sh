#!/bin/bash
# Round-5 single-call latency probe (tools/latency_probe.py), then an A/B of library variants at one
# batch in flight (tools/gpu_r05_ab.sh).  First failure ends the script.
set -o pipefail
OUT=gpurun_out/${1:-r05lat}
mkdir -p $OUT
timeout -k 10 400 python -u -X faulthandler tools/latency_probe.py ${LAT_ARGS:-} > $OUT/latency.jsonl 2> $OUT/latency.err || { tail -20 $OUT/latency.err; exit 1; }
cat $OUT/latency.jsonl
