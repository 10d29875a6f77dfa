#!/bin/bash
# Builds exp/<name>/liblfm.so: the in-tree objects with one source rebuilt
# under extra defines (A/B and timing-probe libraries; LFM_LIB=... selects one).
# usage: scripts/build_variant.sh NAME SOURCE.hip "-DFOO=1 ..."
set -euo pipefail
NAME=$1; SRC=$2; DEFS=${3:-}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/lightfieldmicroscopy_pc-bzip2_amd
OUT=$ROOT/exp/$NAME
mkdir -p "$OUT"
BASE=$(basename "$SRC" .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -w -I"$ROOT/include/lfm" -I"$PKG/csrc" --offload-arch=gfx950 \
    -munsafe-fp-atomics $DEFS -c "$PKG/csrc/$BASE.hip" -o "$OUT/$BASE.o"
OBJS=$(ls "$PKG"/build/*.o | grep -v "/$BASE.o$")
/opt/rocm/bin/hipcc -shared -fPIC -o "$OUT/liblfm.so" $OBJS "$OUT/$BASE.o" -L/opt/rocm/lib -lamdhip64 \
    -lhsa-runtime64 -l:libbz2.so.1.0 -lz -lpthread -Wl,-rpath,/opt/rocm/lib
echo "$OUT/liblfm.so"
