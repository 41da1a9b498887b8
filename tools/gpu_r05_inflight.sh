set -o pipefail
OUT=gpurun_out/r05c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "concurrent or ragged or golden or single" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
for k in 1 2 3 4; do
  timeout -k 10 300 python bench.py --mode verify --steps 30 --warmup 3 --inflight $k --no-cpu-baseline --no-pcie > $OUT/verify_if$k.json 2> $OUT/verify_if$k.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/verify_if$k.json').read().strip().splitlines()[-1]); print('inflight $k', d['value'], d['ms_per_step'], d['default_tables']['value'])"
done
for k in 3 1; do
  timeout -k 10 300 python bench.py --mode verify --steps 30 --warmup 3 --inflight $k --no-cpu-baseline --no-pcie > $OUT/verify_if${k}b.json 2> $OUT/verify_if${k}b.err || exit 1
  python3 -c "import json; d=json.loads(open('$OUT/verify_if${k}b.json').read().strip().splitlines()[-1]); print('inflight $k (again)', d['value'], d['ms_per_step'])"
done
