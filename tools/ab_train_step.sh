set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/ab_step; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "train_step or full_batch or update" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for mode in sep fused; do
    if [ $mode = sep ]; then export SRCNN_BENCH_SEPARATE_UPDATE=1; else unset SRCNN_BENCH_SEPARATE_UPDATE; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/bench_${mode}_$rep.json 2> $OUT/bench_${mode}_$rep.err || exit $?
    python3 -c "import json; d=json.load(open('$OUT/bench_${mode}_$rep.json')); print('$mode rep $rep', round(d['value']), d['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['kernels'].items()}, 'wide', d['wide']['ms_per_step'], {k:round(v['ms_per_step'],4) for k,v in d['wide']['kernels'].items() if k in ('slab_reduce','update_all')})"
  done
done
