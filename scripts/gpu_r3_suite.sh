#!/bin/bash
# Full GPU suite in one process (the driver's invocation) + smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/${1:-suite}
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread \
    > $out/pytest.log 2>&1
rc=$?
grep -E "passed|failed" $out/pytest.log | tail -3
[ $rc -ne 0 ] && { grep -E "FAILED|^E " $out/pytest.log | head -40; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
rc=$?
tail -3 $out/smoke.log
exit $rc
