#!/bin/bash
# Build libsrcnn_hip.so from the kernel sources of a git revision (for
# same-box A/Bs against the working tree):
#   tools/build_rev_variant.sh <name> <rev>  -> cnn-super-resolution_amd/lib/variants/libsrcnn_hip_<name>.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; rev=$2
T=/tmp/srcnn_rev_$name
rm -rf $T && mkdir -p $T
(cd $R && git archive "$rev" include cnn-super-resolution_amd/csrc cnn-super-resolution_amd/Makefile) | tar -x -C $T
P=$R/cnn-super-resolution_amd
O=$T/obj
mkdir -p $O $P/lib/variants
for f in $(cd $T/cnn-super-resolution_amd/csrc/hip && ls *.cpp *.hip); do
  # that revision's per-file flags (FILEFLAGS_<file> := ... in its Makefile)
  ff=$(sed -n "s/^FILEFLAGS_$f := //p" $T/cnn-super-resolution_amd/Makefile)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -munsafe-fp-atomics \
    -Wno-unused-result -I$T/include -I$T/cnn-super-resolution_amd/csrc/hip $ff -x hip \
    -c $T/cnn-super-resolution_amd/csrc/hip/$f -o $O/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/variants/libsrcnn_hip_$name.so $O/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $P/lib/variants/libsrcnn_hip_$name.so from $rev"
