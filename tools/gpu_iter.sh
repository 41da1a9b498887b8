#!/bin/bash
# One iteration of kernel work on the GPU box: the parity tests (TESTS, default the golden-fixture
# suite), then interleaved benches of the previous build (libcoconut_hip_prev.so) and the current one,
# then the fexp phase clocks if the CC_FEXP_PROF build is present.  Each GPU step has its own time limit;
# the first failure ends the script.  Usage: [TESTS=...] [AB_MODE=verify] bash tools/gpu_iter.sh <tag>
set -o pipefail
TAG=${1:-iter}
OUT=gpurun_out/$TAG
MODE=${AB_MODE:-verify}
TESTS=${TESTS:-tests/test_gpu_parity.py}
mkdir -p "$OUT"
echo "[iter] tests $TESTS"
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for k in 1 2; do
  for v in prev cur; do
    lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
    [ $v = prev ] && lib=$(pwd)/coconut-rust_amd/libcoconut_hip_prev.so
    [ -f "$lib" ] || continue
    echo "[iter] bench $v $k"
    COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --mode $MODE --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/${MODE}_$v.$k.json" 2> "$OUT/${MODE}_$v.$k.err" || exit 1
  done
done
if [ -f coconut-rust_amd/libcoconut_hip_prof.so ]; then
  echo "[iter] fexp phases"
  timeout -k 10 300 python -u tools/fexp_phases.py > "$OUT/fexp_phases.json" 2> "$OUT/fexp_phases.err" || exit 1
fi

# optional: one PMC pass per group in PMC_GROUPS (';'-separated counter lists) over one bench step of the
# current build, kernel trace only
if [ -n "${PMC_GROUPS:-}" ]; then
  IFS=';' read -ra GRPS <<< "$PMC_GROUPS"
  i=0
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    echo "[iter] pmc $i: $grp"
    (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d "$OLDPWD/$OUT/pmc$i" -o pmc --output-format csv -- python3 "$OLDPWD/bench.py" --mode $MODE --steps 1 --warmup 0 --no-cpu-baseline --no-pcie > "$OLDPWD/$OUT/pmc$i.log" 2>&1) || exit 1
  done
fi
echo "[iter] pmc done"
