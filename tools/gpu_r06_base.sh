#!/bin/bash
# Round 6 first GPU pass: the full -m gpu suite, smoke, the default bench line (with its same-run SigG1
# leg), and the RLC partials on 1 / 2 slots (pinned staging of the delta seed).  Each step has its own
# time limit; the first failure ends the script.
set -o pipefail
OUT=gpurun_out/${1:-r06a}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('bench', d['value'], d['ms_per_step'], 'sigg1', d.get('sigg1',{}).get('value'), d['kernels']['miller']['ms'], d['kernels']['fexp']['ms'])"
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --mode rlc --steps 20 --warmup 3 --no-cpu-baseline --no-pcie --rlc-inflight $k > "$OUT/rlc_if$k.json" 2> "$OUT/rlc_if$k.err" || { tail -20 "$OUT/rlc_if$k.err"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/rlc_if$k.json'));print('rlc if$k', d['value'], d['ms_per_step'])"
done
