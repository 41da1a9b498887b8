#!/bin/bash
# Round 4: the boundary changes (idempotent set_params / set_verkey, 4 GiB default tables, ordered
# finishes, the config-3 whole workload on one device), smoke, and a default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r04b}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_tables.py tests/test_gpu_rlc.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/verify.json" 2> "$OUT/verify.err" || { tail "$OUT/verify.err"; exit 1; }
timeout -k 10 300 python -u bench.py --mode verify-pervk --steps 5 --warmup 1 > "$OUT/pervk.json" 2> "$OUT/pervk.err" || { tail "$OUT/pervk.err"; exit 1; }
timeout -k 10 300 python -u bench.py --mode verify-pervk-g1 --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/pervk_g1.json" 2> "$OUT/pervk_g1.err" || { tail "$OUT/pervk_g1.err"; exit 1; }
for k in 1 2; do
  for v in prev cur; do
    lib=$(pwd)/coconut-rust_amd/libcoconut_hip.so
    [ $v = prev ] && lib=$(pwd)/coconut-rust_amd/libcoconut_hip_prev.so
    COCONUT_HIP_LIB=$lib timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie > "$OUT/ab_verify_$v.$k.json" 2> "$OUT/ab_verify_$v.$k.err" || exit 1
  done
done
