#!/bin/bash
# Held clocks (in-kernel probe build) of the fused kernels with split-bf16 and
# fp32 layer-1/2 products, same box.   tools/x6_clock.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-x6_clock}
mkdir -p "$OUT"
LIB=$(pwd)/cnn-super-resolution_amd/lib/variants/libsrcnn_hip_probe.so
for a in split f32 split f32; do
  env_a="SRCNN_ARITH=split"; [ $a = f32 ] && env_a="SRCNN_ARITH=f32"
  env $env_a SRCNN_HIP_LIB=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --no-wide --no-forward --steps 20 --warmup 5 \
    > "$OUT/bench_$a.json" 2> "$OUT/bench_$a.err" || { tail "$OUT/bench_$a.err"; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_$a.json'))
print('$a', d['value'], d['ms_per_step'], {k: (v['ms_per_step']) for k, v in d['kernels'].items()})
print('   clocks', {k: r.get('held_clock_ghz') for k, r in d['rooflines'].items()})"
done
