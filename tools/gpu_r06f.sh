set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_pmc.sh r06D --batch 4096 && bash tools/gpu_pmc.sh r06C --config C --batch 4096
