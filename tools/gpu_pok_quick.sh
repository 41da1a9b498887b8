set -o pipefail
mkdir -p gpurun_out/pok1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pok or PoK" > gpurun_out/pok1/pytest.log 2>&1 && \
timeout -k 10 300 python -u bench.py --mode pok --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pok1/bench_pok.json 2>&1
