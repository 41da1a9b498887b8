#!/bin/bash
# Round 4 A/B of two library builds (libcoconut_hip_prev.so vs libcoconut_hip.so) on one box: MODES
# (default verify) alternating prev/cur twice, then the per-verkey bench lines of the current build.
set -o pipefail
OUT=gpurun_out/${1:-r04ab}
MODES=${MODES:-verify}
mkdir -p "$OUT"
for m in $MODES; do
  for k in 1 2; do
    for v in prev cur; do
      lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
      [ $v = prev ] && lib=$(pwd)/coconut-rust_amd/libcoconut_hip_prev.so
      echo "[ab] $m $v $k"
      COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --mode $m --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > "$OUT/${m}_$v.$k.json" 2> "$OUT/${m}_$v.$k.err" || { tail -5 "$OUT/${m}_$v.$k.err"; exit 1; }
    done
  done
done
if [ -n "${EXTRA:-}" ]; then
  echo "[ab] extra: $EXTRA"
  bash -c "$EXTRA" || exit 1
fi
