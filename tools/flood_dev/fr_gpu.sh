# frame-kernel variants beside the product (development): bash tools/flood_dev/fr_gpu.sh TAG lib...
set -uo pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
FDEV_SNR=${FDEV_SNR:--3,0.5} timeout -k 10 400 python -u tools/flood_dev/run_dev.py "$@" > gpurun_out/$TAG/fdev.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/$TAG/fdev.log | tail -40; exit $rc
