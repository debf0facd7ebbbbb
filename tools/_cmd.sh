set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
SESSION_TAG=r01e bash tools/gpu_session.sh pmcmem
