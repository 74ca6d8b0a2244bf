#!/bin/bash
# Build A/B variants of libldpc5g.so into build/alt/<name>.so (compile-time macro / compiler-flag
# switches), for one GPU call to time them side by side:
#   LDPC5G_LIB=build/alt/<name>.so python tools/probe.py layered 4096
set -euo pipefail
rm -rf build/alt
mkdir -p build/alt
build() {   # name, extra flags
  LDPC5G_EXTRA_FLAGS="$2" python -m python_5gtoolbox_amd.build --out "build/alt/$1.so" > "build/alt/$1.log" 2>&1 &
}
build sched_maxilp "-mllvm -amdgpu-sched-strategy=max-ilp"
build misched_maxilp "-mllvm -misched=gcn-max-ilp"
build bias0 "-mllvm -amdgpu-schedule-metric-bias=0"
wait
ls -la build/alt/*.so
