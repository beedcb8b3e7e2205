set -o pipefail
cd $GRAFT_REPO_ROOT
for q in 4 8 16 24; do GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u tools/hwq_probe.py || exit 1; done
