#!/bin/bash
# One SQ counter pass per selection over one verify bench step: the default build, then with the
# environment override $2 (e.g. CC_FEXP=pl).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$(pwd)
OUT=$R/gpurun_out/${1:-pmc_ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
OVR=${2:-CC_MILLER=pl}
for m in new old; do
  echo "[pmc] $m"
  E=(); [ $m = old ] && E=("$OVR")
  env "${E[@]}" timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES -d "$OUT/$m" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline > "$OUT/$m.log" 2>&1 || exit $?
done
echo "[pmc] done"
