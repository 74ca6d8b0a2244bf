set -uo pipefail
OUT=gpurun_out/${TAG:-r01k}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ldpc.py -q -x -k "encode or dlsch" --timeout 120 --timeout-method thread > $OUT/enc_tests_new.log 2>&1; rc=$?; tail -2 $OUT/enc_tests_new.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for lib in python_5gtoolbox_amd/libldpc5g.so build/alt/*.so; do
  for nt in ${NTS:-128}; do
    LDPC5G_ENC_THREADS=$nt LDPC5G_LIB=$PWD/$lib timeout -k 10 120 python -u tools/probe.py encode 4096 16384 > $OUT/probe_$(basename $lib .so)_$nt.log 2>&1 || exit $?
    echo "$lib nt=$nt: $(grep -v amdgpu.ids $OUT/probe_$(basename $lib .so)_$nt.log | tr '\n' ' ')"
  done
done
