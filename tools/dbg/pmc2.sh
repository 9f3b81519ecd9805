set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for L in ""; do
  tag=full; [ -n "$L" ] && tag=x15
  export FRCNN_LIB_PATH=$L
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU --output-format csv -d gpurun_out/r5h/$tag/sq -o run -- python3 tools/ab_roi_pool.py --config cfg2 --variants sort --rounds 1 --iters 3 > gpurun_out/r5h/$tag.sq.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/r5h/$tag/sq2 -o run -- python3 tools/ab_roi_pool.py --config cfg2 --variants sort --rounds 1 --iters 3 > gpurun_out/r5h/$tag.sq2.log 2>&1 || exit 1
  python3 tools/summarize_pmc.py gpurun_out/r5h/$tag roi_pool_fwd_sort > gpurun_out/r5h/$tag.txt; cat gpurun_out/r5h/$tag.txt
done
