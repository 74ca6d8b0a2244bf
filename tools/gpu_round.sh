#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace, encoder A/B probes and
# PMC counter passes.  Usage (from the repo root, via gpurun):  bash tools/gpu_round.sh TAG [steps]
#   steps: comma list of {tests,smoke,bench,trace,rehearse,probe,ab,pmc,calib}; default tests,smoke,bench,trace,probe,pmc.
# Every GPU step has its own time limit.  A test FAILURE (pytest rc 1) does not stop the script;
# a crash, abort or time limit (any other non-zero rc) ends it at once.
set -uo pipefail
TAG=${1:-run}
STEPS=${2:-tests,smoke,bench,trace,probe,pmc}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
has() { [[ ",$STEPS," == *",$1,"* ]]; }
die() { echo "[gpu_round] $1 failed rc=$2 — stopping"; exit "$2"; }

if has tests; then
  echo "[gpu_round] tests"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1
  rc=$?
  tail -5 "$OUT/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then die tests $rc; fi
  if [ $rc -eq 1 ]; then grep -E "^(FAILED|ERROR)|Error" "$OUT/pytest_gpu.log" | head -20; fi
fi
if has smoke; then
  echo "[gpu_round] smoke"
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || die smoke $?
  tail -1 "$OUT/smoke.log"
fi
if has bench; then
  echo "[gpu_round] bench"
  timeout -k 10 420 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; die bench $?; }
  cat "$OUT/bench.json"
fi
if has trace; then
  echo "[gpu_round] rocprof kernel trace"
  cd /tmp
  # each config-3 line alone (the bench's 3 warmup + 20 timed launches; the summary skips the
  # warmups, so the decoder's average is over the launches behind the line's ms_per_step):
  # the headline (float64 flooding, reference-exact), then the float32 layered perf_mode line
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_headline" -o run -- python -u "$ROOT/bench.py" --cpu-seconds 0 --no-extras --no-perf \
      > "$OUT/bench_headline_under_rocprof.json" 2> "$OUT/rocprof_headline.err" || { tail -20 "$OUT/rocprof_headline.err"; die trace $?; }
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_layered" -o run -- python -u "$ROOT/bench.py" --cpu-seconds 0 --no-extras --no-perf --headline layered \
      > "$OUT/bench_layered_under_rocprof.json" 2> "$OUT/rocprof_layered.err" || { tail -20 "$OUT/rocprof_layered.err"; die trace $?; }
  # everything (extras: encoder, flooding, config 4 / 5 chains): per-kernel table
  timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
      python -u "$ROOT/bench.py" --steps 10 --cpu-seconds 0 > "$OUT/bench_under_rocprof.json" 2> "$OUT/rocprof.err" \
      || { tail -20 "$OUT/rocprof.err"; die trace $?; }
  cd "$ROOT"
  python tools/rocpd_summary.py "$OUT/prof_headline" --skip 3 > "$OUT/kernel_stats_headline.csv"
  python tools/rocpd_summary.py "$OUT/prof_layered" --skip 3 > "$OUT/kernel_stats_layered.csv"
  python tools/rocpd_summary.py "$OUT/prof" > "$OUT/kernel_stats.csv"
  cut -c1-150 "$OUT/kernel_stats_headline.csv" | head -6
  cut -c1-150 "$OUT/kernel_stats_layered.csv" | head -6
  cut -c1-150 "$OUT/kernel_stats.csv" | head -12
fi
if has fdev; then
  echo "[gpu_round] float64 flooding variants (build/fdev/*.so)"
  timeout -k 10 300 python -u tools/flood_dev/run_dev.py ${FDEV_LIBS:-build/fdev/*.so} > "$OUT/fdev.log" 2>&1 || { tail -20 "$OUT/fdev.log"; die fdev $?; }
  grep -v amdgpu.ids "$OUT/fdev.log"
fi
if has small; then
  echo "[gpu_round] small-codeblock latency probe"
  timeout -k 10 180 python -u tools/probe_small.py > "$OUT/probe_small.log" 2>&1 || { tail -20 "$OUT/probe_small.log"; die small $?; }
  grep -v amdgpu.ids "$OUT/probe_small.log"
fi
if has rehearse; then
  echo "[gpu_round] 2-rank rehearsal (bench.py --gpus 2 --backend gloo: two ranks on one GPU)"
  timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --no-extras --steps 10 --cpu-seconds 3 \
      > "$OUT/bench_w2_gloo.json" 2> "$OUT/bench_w2_gloo.err" || { tail -20 "$OUT/bench_w2_gloo.err"; die rehearse $?; }
  cat "$OUT/bench_w2_gloo.json"
  timeout -k 10 120 python -u bench.py --gpus 8 --no-extras --cpu-seconds 0 > "$OUT/bench_w8_refused.json" 2> "$OUT/bench_w8_refused.err"
  echo "bare --gpus 8 on one GPU: rc=$? $(cat "$OUT/bench_w8_refused.err")"
fi
if has probe; then
  echo "[gpu_round] throughput probes"
  timeout -k 10 120 python -u tools/probe.py encode 4096 16384 > "$OUT/probe_enc.log" 2>&1 || die probe $?
  timeout -k 10 120 python -u tools/probe.py layered 4096 16384 > "$OUT/probe_layered.log" 2>&1 || die probe $?
  timeout -k 10 120 python -u tools/probe.py flooding64 4096 > "$OUT/probe_flooding64.log" 2>&1 || die probe $?
  grep -hv amdgpu.ids "$OUT"/probe_*.log
fi
if has ab; then
  echo "[gpu_round] decoder A/B builds (build/alt/*.so)"
  for lib in python_5gtoolbox_amd/libldpc5g.so build/alt/*.so; do
    n=$(basename "$lib" .so)
    LDPC5G_LIB=$ROOT/$lib timeout -k 10 240 python -u -m pytest tests/test_gpu_ldpc.py -q -x -k "${AB_TESTS:-layered or packed or z384}" \
        --timeout 120 --timeout-method thread > "$OUT/ab_test_$n.log" 2>&1
    rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then die "ab test $n" $rc; fi
    LDPC5G_LIB=$ROOT/$lib timeout -k 10 120 python -u tools/probe.py ${AB_PROBE:-layered} 4096 16384 > "$OUT/ab_probe_$n.log" 2>&1 || die "ab probe $n" $?
    echo "$n: tests $(tail -1 "$OUT/ab_test_$n.log") | $(grep -v amdgpu.ids "$OUT/ab_probe_$n.log" | tr '\n' ' ')"
  done
fi
if has pmc; then
  echo "[gpu_round] PMC passes"
  cd /tmp
  i=0
  for ctr in "FETCH_SIZE" "WRITE_SIZE" \
             "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"; do
    i=$((i + 1))
    # PMC_ARGS: the profiled program's arguments (default: the headline bench)
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/pmc$i" -o run -- \
        python -u ${PMC_ARGS:-"$ROOT/tools/pmc_probe.py" 3} \
        > "$OUT/pmc$i.json" 2> "$OUT/pmc$i.err" || { tail -5 "$OUT/pmc$i.err"; cd "$ROOT"; die "pmc $ctr" $?; }
  done
  cd "$ROOT"
  python tools/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json" && cat "$OUT/pmc_summary.json"
fi
if has icache; then
  echo "[gpu_round] instruction-cache counters (tools/pmc_probe.py)"
  cd /tmp
  i=0
  for ctr in "SQC_ICACHE_REQ SQC_ICACHE_MISSES" "SQC_ICACHE_HITS SQC_ICACHE_MISSES_DUPLICATE" "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
    i=$((i + 1))
    timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d "$OUT/icache$i" -o run -- \
        python -u "$ROOT/tools/pmc_probe.py" 2 > "$OUT/icache$i.log" 2>&1 || { tail -5 "$OUT/icache$i.log"; cd "$ROOT"; die "icache $ctr" $?; }
  done
  cd "$ROOT"
  mkdir -p "$OUT/icache_all" && cp -r "$OUT"/icache[0-9]* "$OUT/icache_all/" 2>/dev/null
  python - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for f in sorted(glob.glob(out + "/icache[0-9]*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("ldpc5g_impl::", "").replace("(anonymous namespace)::", "")
        if "ldpc" not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k[:70], {c: f"{x:.4g}" for c, x in sorted(v.items())})
PY
fi
if has calib; then
  echo "[gpu_round] FETCH_SIZE / WRITE_SIZE calibration (tools/microbench/fetch_calib: 1 GiB per kernel)"
  cd /tmp
  timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/calib_fetch" -o run -- \
      "$ROOT/tools/microbench/fetch_calib" > "$OUT/calib_fetch.log" 2>&1 || { tail -5 "$OUT/calib_fetch.log"; cd "$ROOT"; die "calib fetch" $?; }
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/calib_write" -o run -- \
      "$ROOT/tools/microbench/fetch_calib" > "$OUT/calib_write.log" 2>&1 || { tail -5 "$OUT/calib_write.log"; cd "$ROOT"; die "calib write" $?; }
  cd "$ROOT"
  python tools/microbench/fetch_calib.py "$OUT" > "$OUT/fetch_calib.json" && cat "$OUT/fetch_calib.json"
fi
echo "[gpu_round] done"
