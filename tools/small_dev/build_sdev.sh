#!/bin/bash
# Build the small-codeblock decoder dev harness: build/sdev/<name>.so for each "name:flags" argument.
#   bash tools/small_dev/build_sdev.sh base: base_ts:-DLDPC5G_SMALL_TS
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
mkdir -p "$ROOT/build/sdev"
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared \
    -I"$ROOT/include" -I"$ROOT/python_5gtoolbox_amd/csrc" $flags "$ROOT/tools/small_dev/sdev.hip" \
    -o "$ROOT/build/sdev/$name.so" &
done
wait
