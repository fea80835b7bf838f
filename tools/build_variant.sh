#!/bin/bash
# Build librecsys_hip.$NAME.so: SRC (a csrc/*.hip translation unit) recompiled with extra FLAGS, linked with the
# other in-tree objects (run the normal build first).  For A/B timing with RS_LIB_VARIANT=$NAME (tools/gpu.sh ab).
#   NAME=p1 SRC=rowchain.hip FLAGS="-DRC_HEAD_PREFETCH=1" bash tools/build_variant.sh
set -e
cd "$(dirname "$0")/.."
PKG=recommender-baseline-model_amd
OBJ=$PKG/csrc/build
mkdir -p /tmp/rsvar
# SRC may name several translation units (space-separated)
vobjs=""
objs=$(ls $OBJ/*.o)
for f in $SRC; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -I include -I $PKG/csrc $FLAGS \
    -c $PKG/csrc/$f -o /tmp/rsvar/$f.$NAME.o
  vobjs="$vobjs /tmp/rsvar/$f.$NAME.o"
  objs=$(echo "$objs" | grep -v "/$f.o$")
done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs $vobjs -o $PKG/librecsys_hip.$NAME.so
echo $PKG/librecsys_hip.$NAME.so
