set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python scripts/diag_c1.py 0.15 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python scripts/diag_c1.py 0.0 2>&1 | grep -v amdgpu.ids
