#!/bin/bash
# Variant builds of the multi-workgroup flooding kernel (development tool): only
# ldpc5g_dec_split.hip is recompiled with the variant's flags, linked with the product objects.
#   bash tools/split_dev/build.sh NAME "-DLDPC5G_SPLIT_TS ..."   -> build/alt/split_NAME.so
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
NAME=$1; shift
OUT=$ROOT/build/split_dev; mkdir -p "$OUT" "$ROOT/build/alt"
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-result -I"$ROOT/include" \
    -I"$ROOT/python_5gtoolbox_amd/csrc" $@ -c "$ROOT/python_5gtoolbox_amd/csrc/ldpc5g_dec_split.hip" -o "$OUT/$NAME.o"
objs=$(ls "$ROOT"/build/obj/*.hip.o | grep -v ldpc5g_dec_split)
$HIPCC --offload-arch=gfx950 -shared -fPIC $objs "$OUT/$NAME.o" -o "$ROOT/build/alt/split_$NAME.so"
echo "built build/alt/split_$NAME.so"
