cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03_s512
for b in 512 1024; do
timeout -k 10 200 python bench.py --batch $b --no-cpu-baseline --no-wide --no-forward --steps 200 --warmup 50 > gpurun_out/r03_s512/b$b.json 2> gpurun_out/r03_s512/b$b.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/r03_s512/b$b.json')); print($b, d['ms_per_step'], {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
