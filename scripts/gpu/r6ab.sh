set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6ab; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -k "sequence or run_twice" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
