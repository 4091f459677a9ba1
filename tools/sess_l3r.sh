# l3r A/B session: parity + timing of the variants named on the command line
cd $GRAFT_REPO_ROOT
V=${@:-"l3r l3old"}
libs=""; for v in $V; do libs="$libs cnn-super-resolution_amd/lib/variants/libsrcnn_hip_$v.so"; done
bash tools/ab_step.sh ab_${TAG:-l3r} $libs || exit $?
for v in ${TIMING:-}; do
  echo "== $v"
  SRCNN_HIP_LIB=$PWD/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_$v.so timeout -k 10 120 python tools/l3_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
