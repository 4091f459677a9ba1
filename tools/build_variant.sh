#!/bin/bash
# Build a diagnostic variant of libsrcnn_hip.so with extra compile flags:
#   tools/build_variant.sh <name> [-DFLAG ...]  -> cnn-super-resolution_amd/lib/variants/libsrcnn_hip_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/cnn-super-resolution_amd
name=$1; shift
O=$P/build/variant_$name
mkdir -p $O $P/lib/variants
for f in $(cd $P/csrc/hip && ls *.cpp *.hip); do
  # the Makefile's per-file flags (FILEFLAGS_<file> := ...)
  ff=$(sed -n "s/^FILEFLAGS_$f := //p" $P/Makefile)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -munsafe-fp-atomics \
    -Wno-unused-result -I$R/include -I$P/csrc/hip $ff "$@" -x hip -c $P/csrc/hip/$f -o $O/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libsrcnn_hip_$name.so $O/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo built $P/lib/variants/libsrcnn_hip_$name.so
