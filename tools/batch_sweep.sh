cd "$GRAFT_REPO_ROOT"
for b in 4096 2048 1024 512 256; do
  timeout -k 10 120 python bench.py --batch $b --steps 40 --warmup 5 --no-cpu-baseline --no-wide --no-forward > gpurun_out/bs_$b.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.load(open('gpurun_out/bs_$b.json')); b=$b
print(b, round(d['value']), d['ms_per_step'], {k: round(v['ms_per_step']*4096/b,4) for k,v in d['kernels'].items()})"
done
