#!/bin/bash
# Same-box A/B (bench only): the previous library build (libcoconut_hip_prev.so) against the current
# one, interleaved, after the GPU suite of the current build.  Usage: [AB_MODE=rlc] bash tools/gpu_ab_ll.sh <tag>
set -o pipefail
TAG=${1:-ab}
OUT=gpurun_out/$TAG
MODE=${AB_MODE:-verify}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
for k in 1 2; do
  for v in prev cur; do
    lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
    [ $v = prev ] && lib=$(pwd)/coconut-rust_amd/libcoconut_hip_prev.so
    echo "[ab] $v $k"
    COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --mode $MODE --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${MODE}_$v.$k.json" 2>&1 || exit 1
  done
done
echo "[ab] done"
