#!/bin/bash
# Variant build of ONE translation unit (development tool): csrc/TU recompiled with the given
# flags, linked with the product objects of every other TU.
#   bash tools/split_dev/build_tu.sh TU.hip NAME "-D..."   -> build/alt/NAME.so
#   (SRC=dir: compile the TU from dir/python_5gtoolbox_amd/csrc, e.g. a `git archive` of another commit)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
TU=$1; NAME=$2; shift 2
OUT=$ROOT/build/split_dev; mkdir -p "$OUT" "$ROOT/build/alt"
HIPCC=/opt/rocm/bin/hipcc
EXTRA=""; case "$TU" in ldpc5g_dec_l.hip|ldpc5g_dec_l_dead.hip) EXTRA="-fno-slp-vectorize";; esac
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Wno-unused-result $EXTRA -I"$ROOT/include" \
    -I"${SRC:-$ROOT}/python_5gtoolbox_amd/csrc" $@ -c "${SRC:-$ROOT}/python_5gtoolbox_amd/csrc/$TU" -o "$OUT/$NAME.o"
objs=$(ls "$ROOT"/build/obj/*.hip.o | grep -v "/$TU.o")
$HIPCC --offload-arch=gfx950 -shared -fPIC $objs "$OUT/$NAME.o" -o "$ROOT/build/alt/$NAME.so"
echo "built build/alt/$NAME.so"
