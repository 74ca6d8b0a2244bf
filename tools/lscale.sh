# iteration scaling of the decoders + layered parity tests (development probe)
set -uo pipefail
OUT=gpurun_out/${1:-r03e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest_ldpc.log 2>&1
rc=$?; tail -3 $OUT/pytest_ldpc.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for L in 1 2 4 8; do PROBE_L=$L timeout -k 10 120 python -u tools/probe.py layered 4096 16384 || exit $?; done > $OUT/lscale.txt 2>&1
for L in 1 8; do PROBE_L=$L timeout -k 10 120 python -u tools/probe.py flooding64 4096 || exit $?; done >> $OUT/lscale.txt 2>&1
PROBE_SNR=1 timeout -k 10 120 python -u tools/probe.py layered 4096 16384 >> $OUT/lscale.txt 2>&1
grep -v amdgpu.ids $OUT/lscale.txt
if [ "${WITH_BENCH:-0}" = 1 ]; then
  timeout -k 10 420 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 3; }
  python -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step']); [print(k, v) for k, v in d.get('extras', {}).items()]" | cut -c1-400
fi
