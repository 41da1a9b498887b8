#!/bin/bash
# Round-5 spread point arithmetic (curve_wide_lz.h) in the one-wave PoK / per-credential-verkey preps:
# their path-agreement tests and goldens, optionally the whole -m gpu suite (FULL=1), then the bench
# lines whose single-call latency legs they shorten.
set -o pipefail
OUT=gpurun_out/${1:-r05s}
mkdir -p $OUT
T="python -u -X faulthandler -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $T tests/test_gpu_parity.py -k "pok or pervk or per_credential" > $OUT/pytest_pok.log 2>&1 || { tail -30 $OUT/pytest_pok.log; exit 1; }
tail -1 $OUT/pytest_pok.log
if [ "${FULL:-0}" = 1 ]; then
  timeout -k 10 600 $T tests > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
run() {  # name, args
  timeout -k 10 400 python -X faulthandler bench.py $2 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d.get('kernels', {}).items()}, json.dumps(d.get('latency')))"
}
for m in ${MODES:-pok pok-g1}; do
  case $m in
    pervk) run pervk "--mode verify-pervk --steps 10 --warmup 2 --no-cpu-baseline" ;;
    pervk-g1) run pervk-g1 "--mode verify-pervk-g1 --steps 10 --warmup 2 --no-cpu-baseline" ;;
    *) run $m "--mode $m --steps 10 --warmup 2 --no-cpu-baseline" ;;
  esac
done
