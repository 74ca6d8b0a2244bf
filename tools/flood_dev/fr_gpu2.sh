# frame-kernel variants on plain and on rate-matched (dead extension columns) inputs (development)
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
FDEV_SNR=-3 timeout -k 10 300 python -u tools/flood_dev/run_dev.py "$@" > gpurun_out/$TAG/fdev_plain.log 2>&1 || { tail -20 gpurun_out/$TAG/fdev_plain.log; exit 1; }
grep -v amdgpu.ids gpurun_out/$TAG/fdev_plain.log
FDEV_SNR=-3 FDEV_DEADCOLS=30 timeout -k 10 300 python -u tools/flood_dev/run_dev.py "$@" > gpurun_out/$TAG/fdev_dead30.log 2>&1 || { tail -20 gpurun_out/$TAG/fdev_dead30.log; exit 1; }
echo "dead 30:"; grep -v amdgpu.ids gpurun_out/$TAG/fdev_dead30.log
