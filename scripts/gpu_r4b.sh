#!/bin/bash
# Round 4: the whole GPU suite in one process (the driver's invocation) + smoke.
# Usage: gpu_r4b.sh <outdir-name>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/${1:-r4b}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $O/pytest.log | tail -2
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $O/pytest.log | head -40; exit $rc; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
