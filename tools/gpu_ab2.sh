#!/bin/bash
# Interleaved A/B of two library builds on one box (bench only).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd); OUT=$R/gpurun_out/ab2; mkdir -p "$OUT"
for k in 1 2; do
for v in prev cur; do
  lib=$R/coconut-rust_amd/libcoconut_hip.so; [ $v = prev ] && lib=$R/coconut-rust_amd/libcoconut_hip_prev.so
  echo "[ab2] $v $k"
  COCONUT_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/$v.$k.json" 2>&1
done; done
echo "[ab2] done"
