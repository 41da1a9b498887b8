#!/bin/bash
# Rehearsal of bench.py's multi-rank path on a one-GPU box: two ranks under torch.distributed.run over
# gloo sharing the GPU (barriers, max over ranks, the sigg1 leg under a process group, the RLC all-gather
# through host memory).  Not a scaling measurement: both ranks share one GPU.
set -o pipefail
OUT=gpurun_out/${1:-r06_rehearse}
mkdir -p "$OUT"
timeout -k 10 900 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > "$OUT/verify_gloo2.json" 2> "$OUT/verify_gloo2.err" || { tail -30 "$OUT/verify_gloo2.err"; exit 1; }
tail -c 600 "$OUT/verify_gloo2.json"; echo
timeout -k 10 600 python -u bench.py --mode rlc --gpus 2 --backend gloo --steps 5 --warmup 1 --no-cpu-baseline --no-pcie > "$OUT/rlc_gloo2.json" 2> "$OUT/rlc_gloo2.err" || { tail -30 "$OUT/rlc_gloo2.err"; exit 1; }
tail -c 400 "$OUT/rlc_gloo2.json"; echo
