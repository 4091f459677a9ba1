#!/bin/bash
# A/B the phases of the l3_delta kernel (diagnostics; results are not valid outputs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/${1:-abl}
for a in 0 1 2 4 7 0; do
  SRCNN_ABLATE_L3=$a timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/${1:-abl}/ablate_$a.json 2>/dev/null || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/${1:-abl}/ablate_$a.json')); print('ablate=$a', {k:v['ms_per_step'] for k,v in d['kernels'].items()})"
done
