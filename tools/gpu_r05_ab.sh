#!/bin/bash
# Round-5 same-box A/B of library variants (coconut-rust_amd/libcoconut_hip_<v>.so, built from modified
# copies of csrc/) against the current build: config 2 at one batch in flight, alternating, twice.
set -o pipefail
OUT=gpurun_out/${1:-r05ab}
VARIANTS=${VARIANTS:-"vA vB"}
mkdir -p $OUT
for k in 1 2; do
  for v in cur $VARIANTS; do
    lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
    [ $v = cur ] || lib=$(pwd)/coconut-rust_amd/libcoconut_hip_$v.so
    COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --mode ${MODE:-verify} --steps 20 --warmup 3 --inflight 1 --no-cpu-baseline --no-pcie > $OUT/${v}.$k.json 2> $OUT/${v}.$k.err || { tail -5 $OUT/${v}.$k.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${v}.$k.json').read().strip().splitlines()[-1]); print('$v $k', d['value'], {k_: v_['ms'] for k_, v_ in d['kernels'].items()})"
  done
done
