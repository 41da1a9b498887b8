#!/bin/bash
# Round-5: verify twice (box variance check against earlier runs), then the PoK and per-credential-verkey
# lines with their new single-call latency legs.  First failure ends.
set -o pipefail
OUT=gpurun_out/${1:-r05l}
mkdir -p $OUT
run() {  # name, args
  timeout -k 10 400 python -X faulthandler bench.py $2 > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d.get('kernels', {}).items()}, json.dumps(d.get('latency')))"
}
run verify "--steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
run verify_b "--steps 20 --warmup 3 --no-cpu-baseline --no-pcie"
run pok "--mode pok --steps 10 --warmup 2 --no-cpu-baseline"
run pervk "--mode verify-pervk --steps 10 --warmup 2 --no-cpu-baseline"
