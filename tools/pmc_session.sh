#!/bin/bash
# PMC counter passes over a short bench run (one rocprofv3 run per pass,
# --pmc combined with --kernel-trace only).  Output: gpurun_out/<tag>/pmc/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/${1:-pmc}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
have() { grep -qw "$1" "$OUT/counters.txt"; }
run_pass() {
  local name=$1; shift
  local list=()
  for c in "$@"; do have "$c" && list+=("$c"); done
  [ ${#list[@]} -eq 0 ] && { echo "pass $name: no counters available"; return 0; }
  echo "pass $name: ${list[*]}"
  timeout -k 10 300 rocprofv3 --pmc "${list[@]}" --kernel-trace --output-format csv -d "$OUT/$name" -o run \
    -- python3 "$ROOT/bench.py" --steps ${PMC_STEPS:-3} --warmup 1 --no-cpu-baseline ${PMC_BENCH_ARGS:-} > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
PASSES=${PMC_PASSES:-fetch write sq1 sq2 sq3 tcc}
want() { case " $PASSES " in *" $1 "*) return 0;; esac; return 1; }
want fetch && { run_pass fetch FETCH_SIZE || exit $?; }
want write && { run_pass write WRITE_SIZE || exit $?; }
want sq1 && { run_pass sq1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT || exit $?; }
want sq2 && { run_pass sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR || exit $?; }
want sq3 && { run_pass sq3 SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_MFMA SQ_LDS_UNALIGNED_STALL SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_VALU_FMA_F32 || exit $?; }
want tcc && { run_pass tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum || exit $?; }
echo done
