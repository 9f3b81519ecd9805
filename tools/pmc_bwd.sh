# PMC passes (one counter group per run) over tools/ab_roi_pool_bwd.py with one
# backward variant, summarised for its kernel:
#   bash tools/pmc_bwd.sh OUTDIR VARIANT KERNEL_SUBSTRING     (VARIANT: lead | b1 | b2 | ...)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=$1; VAR=$2; KERN=$3
mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 tools/ab_roi_pool_bwd.py --paths "$VAR" --rounds 1 --iters 3 > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU && \
run sq2 SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
run sq3 SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_SENDMSG SQ_INSTS_LDS && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
python3 tools/summarize_pmc.py "$OUT" "$KERN" --config cfg5 > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
