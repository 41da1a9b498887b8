#!/bin/bash
# PMC passes over one bench step (separate rocprofv3 run per counter group; kernel-trace only).
# BENCH_ARGS selects the bench mode (default: the config-2 verify step).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=${PMC_OUT:-$R/gpurun_out/pmc}
BARGS=${BENCH_ARGS:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_WAIT_ANY" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  echo "[pmc] pass $i: $grp"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$OUT/p$i" -o pmc --output-format csv -- python3 "$R/bench.py" $BARGS --steps 1 --warmup 0 --no-cpu-baseline --no-pcie --no-sigg1 > "$OUT/p$i.log" 2>&1
done
echo "[pmc] done"
