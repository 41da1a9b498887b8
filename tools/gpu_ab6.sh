#!/bin/bash
# Round-6 A/B on one GPU box: the parity tests (TESTS) on the current build, then the previous build
# (libcoconut_hip_prev.so, tools/build_prev.sh) and the current one alternating, twice, for every mode in
# MODES and every argument set in ARGS_LIST (';'-separated), then (PROF=1) rocprofv3 kernel stats and the
# PMC passes of the current build for each mode at one batch in flight.  Each GPU step has its own time
# limit; the first failure ends the script.
#   TESTS="tests/test_gpu_parity.py" KEXPR="pervk" MODES="verify-pervk" ARGS_LIST="--inflight 2;--inflight 1" \
#     PROF=1 bash tools/gpu_ab6.sh <tag>
# PREV_ENV="COCONUT_VKAGG_BA=0": the prev side is the current build with that environment (a runtime switch)
set -o pipefail
TAG=${1:-ab}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
R=$(pwd)
export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  echo "[ab] tests $TESTS"
  KX=()
  [ -n "${KEXPR:-}" ] && KX=(-k "$KEXPR")
  timeout -k 10 900 python -u -m pytest $TESTS "${KX[@]}" -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
IFS=';' read -ra ARGSETS <<< "${ARGS_LIST:-}"
[ ${#ARGSETS[@]} -eq 0 ] && ARGSETS=("")
for m in ${MODES:-verify}; do
  a=0
  for args in "${ARGSETS[@]}"; do
    a=$((a+1))
    for k in 1 2; do
      for v in prev cur; do
        lib=$R/coconut-rust_amd/libcoconut_hip.so
        penv=()
        if [ $v = prev ]; then
          # PREV_ENV="VAR=value": the prev side is the current build under that environment
          if [ -n "${PREV_ENV:-}" ]; then penv=($PREV_ENV); else lib=$R/coconut-rust_amd/libcoconut_hip_prev.so; fi
        fi
        [ -f "$lib" ] || continue
        f="$OUT/${m}_a${a}_${v}.$k.json"
        env "${penv[@]}" COCONUT_HIP_LIB=$lib timeout -k 10 400 python -u bench.py --mode $m --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline --no-pcie --no-sigg1 $args > "$f" 2> "${f%.json}.err" || { tail -20 "${f%.json}.err"; exit 1; }
        python3 -c "import json,sys;d=json.load(open('$f'));k=d.get('kernels',{});print('[ab] $m [$args] $v $k', d['value'], d['ms_per_step'], {x:(y.get('ms') if isinstance(y, dict) else y) for x,y in k.items()})"
      done
    done
  done
  if [ "${PROF:-0}" = 1 ]; then
    P=$OUT/prof_$m
    mkdir -p "$P"
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$P/prof" -o bench --output-format csv -- python3 "$R/bench.py" --mode $m --steps 20 --warmup 2 --no-cpu-baseline --no-pcie --no-sigg1 --inflight 1 > "$P/prof_bench.json" 2> "$P/prof.err") || { echo "rocprof failed"; exit 1; }
    PMC_OUT="$P/pmc" BENCH_ARGS="--mode $m" bash tools/pmc_round.sh > "$P/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
    python3 tools/pmc_summary.py "$P/pmc" "$P/pmc_summary.json" > "$P/pmc_summary.log" 2>&1
    echo "[ab] prof $m done"
  fi
done
echo "[ab] done"
