# PMC of the pair and wave RoIPool forward kernels at cfg2 (SQ groups only).
set -u
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-r3h}
mkdir -p "$OUT"
bash tools/pmc_roi_pool.sh "$OUT/pmc_pair" pair cfg2 || exit 1
bash tools/pmc_roi_pool.sh "$OUT/pmc_wave" wave cfg2 || exit 1
