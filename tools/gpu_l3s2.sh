set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "train_step or l3_kernels or full_batch" > gpurun_out/l3s2_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/l3s2_pytest.log; [ $rc -eq 0 ] || exit $rc
SRCNN_HIP_LIB=$PWD/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_l3st.so timeout -k 10 120 python tools/l3s_timing.py 4096 || exit $?
SRCNN_HIP_LIB=$PWD/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_l3st.so timeout -k 10 120 python tools/l3s_timing.py 512 || exit $?
bash tools/ab_l3.sh ab_l3s_v2 || exit $?
mkdir -p gpurun_out/ab_l3s_v2td6
for b in 4096 512; do SRCNN_L3=stream SRCNN_HIP_LIB=$PWD/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_l3td6.so timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-wide --no-forward > gpurun_out/ab_l3s_v2td6/b$b.json 2>/dev/null || exit $?; python3 -c "import json; d=json.load(open('gpurun_out/ab_l3s_v2td6/b$b.json')); print('td6', $b, d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"; done
mkdir -p gpurun_out/ab_d1cparts
for p in 2 1 2 1; do SRCNN_D1C_PARTS=$p timeout -k 10 200 python bench.py --batch 512 --no-cpu-baseline --no-wide --no-forward --steps 200 --warmup 50 > gpurun_out/ab_d1cparts/p$p.json 2>/dev/null || exit $?; python3 -c "import json; d=json.load(open('gpurun_out/ab_d1cparts/p$p.json')); print('d1c parts', $p, d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"; done
bash tools/ab_fwdq.sh ab_fwdq_v2 || exit $?
