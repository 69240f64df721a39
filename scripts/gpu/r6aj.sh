set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6aj; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u scripts/w1q28.py > $O/w1q.json 2> $O/w1q.err || { tail -5 $O/w1q.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/w1q.json')); print('w1q', d['frac'], d['avg_launch_ms'])"
