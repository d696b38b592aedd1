set -o pipefail
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r6b.sh; echo "profile rc=$?"
bash scripts/gpu_r6c.sh
