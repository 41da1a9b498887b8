#!/bin/bash
# Copy a gpu_modes_prof.sh run (gpurun_out/<tag>/<mode>/) into the committed evidence layout that
# bench.py's kernel_pmc_report reads: profiles/<round>/modes/<mode>/{bench.json, rocprof_kernel_stats.csv,
# pmc_summary.json}.  Usage: tools/collect_modes.sh <tag> <round>
set -euo pipefail
TAG=$1; RND=$2
for d in gpurun_out/$TAG/*/; do
  m=$(basename "$d")
  out=profiles/$RND/modes/$m
  mkdir -p "$out"
  stats=$(find "$d/prof" -name "*kernel_stats.csv" | head -1)
  [ -n "$stats" ] && cp "$stats" "$out/rocprof_kernel_stats.csv"
  [ -f "$d/pmc_summary.json" ] && cp "$d/pmc_summary.json" "$out/pmc_summary.json"
  [ -f "$d/prof_bench.json" ] && tail -1 "$d/prof_bench.json" > "$out/bench.json"
  echo "$m: $(ls "$out" | tr '\n' ' ')"
done
