# PMC passes (one counter group per run) over the RoIPool A/B driver, or over
# the bench itself when VAR=bench.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmc}
VAR=${2:-sorted}
CFG=${3:-cfg2}
mkdir -p "$OUT"
run() {  # name counters...
  local name=$1; shift
  if [ "$VAR" = bench ]; then
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 bench.py --config "$CFG" --steps 3 --warmup 1 --cpu-seconds 0 > "$OUT/$name.log" 2>&1
  else
    timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 tools/ab_roi_pool.py --config "$CFG" --variants "$VAR" --rounds 1 --iters 3 > "$OUT/$name.log" 2>&1
  fi
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU && \
run sq2 SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE
