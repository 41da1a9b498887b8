"""Summarise tools/gpu_iter.sh output: value, ms/step and per-phase ms of each bench line."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        lines = [l for l in open(f).read().strip().split("\n") if l.startswith("{")]
        x = json.loads(lines[-1])
    except (ValueError, IndexError):
        continue
    if "value" in x:
        k = x.get("kernels", {})
        ph = {n: (v["ms"] if isinstance(v, dict) else v) for n, v in k.items()} if isinstance(k, dict) else k
        print(os.path.basename(f), x["value"], x.get("ms_per_step"), ph)
    elif "phases" in x:
        print(os.path.basename(f), round(x["total_clk_per_wave"]), {n: v["frac"] for n, v in x["phases"].items()})
