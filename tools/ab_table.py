"""Summarise an A/B directory of bench JSON lines (tools/gpu_r04_ab.sh): value and phase times per
mode and build, both runs."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    try:
        j = json.load(open(f))
    except Exception as e:  # noqa: BLE001
        print(os.path.basename(f), "unreadable", e)
        continue
    ph = j.get("phase_ms") or {}
    kern = {k.split("(")[0][-28:]: round(v.get("avg_ms", 0), 3) for k, v in (j.get("kernels") or {}).items()} \
        if isinstance(j.get("kernels"), dict) else {}
    print(f"{os.path.basename(f):28s} {j['value']:>12.1f} {j['ms_per_step']:8.3f} ms  {ph}  {kern if kern else ''}")
