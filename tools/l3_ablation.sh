set -u
mkdir -p gpurun_out/l3abl
for v in l3t l3t_nost l3t_nod2 l3t_nogw3 l3t_nodma l3t_nostd2; do
  echo "== $v"
  SRCNN_HIP_LIB=$PWD/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_$v.so timeout -k 10 120 python tools/l3_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
