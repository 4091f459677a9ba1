set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/w1; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_wide_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/wide.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 $OUT/wide.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-forward > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -5 $OUT/bench.err
exit $rc
