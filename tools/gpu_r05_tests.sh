mkdir -p gpurun_out/r05a
timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_flows.py tests/test_gpu_rlc.py tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r05a/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r05a/pytest.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err
  rc2=$?
  tail -c 600 gpurun_out/r05a/bench.json
  exit $rc2
fi
exit $rc
