#!/bin/bash
# Verkey-table window width sweep (cc_set_table_bits): config 2 / 3 / 5 bench lines at each width.
# Each GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
OUT=gpurun_out/${1:-vkbits}
shift || true
BITS=${*:-16 20 22}
mkdir -p "$OUT"
for b in $BITS; do
  for m in verify rlc pok; do
    echo "[vkbits] $m $b"
    timeout -k 10 300 python -u bench.py --mode $m --steps 5 --warmup 1 --no-cpu-baseline --no-pcie --vk-bits $b > "$OUT/${m}_$b.json" 2> "$OUT/${m}_$b.err"
  done
done
echo "[vkbits] done"
