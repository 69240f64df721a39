#!/bin/bash
# Round 4: W-1Q far-target sweep, then the profiles (rocprof stats + PMC).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=${1:-r4f}
bash scripts/gpu_r4_w1q.sh $O/w1q || exit 1
bash scripts/gpu_r4_prof.sh $O/prof
