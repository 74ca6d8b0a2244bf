#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel-trace summary.
# Usage (from the repo root, via gpurun):  bash tools/gpu_round.sh [tag]
# Every GPU step has its own time limit; the first failure ends the script.
set -euo pipefail
TAG=${1:-run}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
echo "[gpu_round] tests"
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
echo "[gpu_round] smoke"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -2 "$OUT/smoke.log"
echo "[gpu_round] bench"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
echo "[gpu_round] rocprof kernel trace"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python -u "$ROOT/bench.py" --steps 10 --cpu-seconds 0 > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err"
cd "$ROOT"
find "$OUT/prof" -name '*kernel_stats.csv' -exec head -8 {} \;
