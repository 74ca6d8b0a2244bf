#!/bin/bash
# Kernel-trace A/B of libldpc5g builds over the full bench (dev tool):  bash tools/ab_trace.sh TAG PATTERN
# For each of python_5gtoolbox_amd/libldpc5g.so and build/alt/*.so: rocprofv3 kernel trace of
# bench.py --steps 4, then the per-kernel stats lines matching PATTERN.
set -uo pipefail
TAG=$1; PAT=$2; ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
for lib in python_5gtoolbox_amd/libldpc5g.so build/alt/*.so; do
  n=$(basename "$lib" .so)
  cd /tmp
  LDPC5G_LIB=$ROOT/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$n" -o run -- \
      python -u "$ROOT/bench.py" --steps 4 --cpu-seconds 0 > "$OUT/$n.json" 2> "$OUT/$n.err" || { tail -5 "$OUT/$n.err"; exit 3; }
  cd "$ROOT"
  echo "== $n"; grep -E "$PAT" "$OUT/$n/run_kernel_stats.csv" | cut -c1-160
done
