# which MFMA / busy counters this gfx950 rocprofv3 offers
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
grep -i "mfma\|BUSY_CU\|GRBM_GUI\|VALU_BUSY\|SQ_BUSY" gpurun_out/pmc_avail.txt | head -60
