# Wide-net A/B of library builds (tools/build_variant.sh, one per source tree
# or flag set): wide parity + bench per variant, then the HBM-byte
# passes (FETCH_SIZE, WRITE_SIZE) per variant.  Variants as arguments.
cd $GRAFT_REPO_ROOT
V=${@:-"nohalo halo"}
TAG=${TAG:-wg2}
libs=""; for v in $V; do libs="$libs cnn-super-resolution_amd/lib/variants/libsrcnn_hip_$v.so"; done
bash tools/ab_wide.sh ab_$TAG $libs || exit $?
for v in $V; do
  SRCNN_HIP_LIB=$PWD/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_$v.so PMC_PASSES="fetch write" \
    PMC_BENCH_ARGS="--no-forward" bash tools/pmc_session.sh ab_$TAG/$v || exit $?
  python3 profiles/pmc_summary.py gpurun_out/ab_$TAG/$v/pmc gpurun_out/ab_$TAG/pmc_$v.json | grep -E "wide_grad2|wide_" || exit 1
done
