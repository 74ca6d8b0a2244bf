# dev round: GPU tests, phase timestamps, probes (tools/lscale.sh), optional bench
set -uo pipefail
TAG=${1:-r03x}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -2 $OUT/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" $OUT/pytest_gpu.log | head; exit 1; fi
(for L in 1 8; do
  LDPC5G_LIB=build/alt/lay_ts.so timeout -k 10 120 python -u tools/ts_probe.py layered 4096 $L || exit $?
  LDPC5G_LIB=build/alt/flood_ts.so timeout -k 10 120 python -u tools/ts_probe.py flooding64 4096 $L || exit $?
done) 2>&1 | grep -v amdgpu.ids > $OUT/ts.txt || exit 2
grep -E "^(layered|flooding)|syndrome|prologue|store" $OUT/ts.txt
for w in layered flooding64; do timeout -k 10 120 python -u tools/probe.py $w 4096 || exit 3; done 2>&1 | grep -v amdgpu.ids
PROBE_SNR=1 timeout -k 10 120 python -u tools/probe.py layered 4096 2>&1 | grep -v amdgpu.ids
if [ "${WITH_BENCH:-0}" = 1 ]; then
  timeout -k 10 420 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 4; }
  python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step']); [print(k, str(v)[:300]) for k, v in d.get('extras', {}).items()]"
fi
