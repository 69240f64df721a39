set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r6aa; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_relayout_gpu.py tests/test_cpp_api.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 900 python -u bench.py --steps 5 --warmup 1 --extras w_hc_seq --no-1q28 --no-batch16 --cpu-budget 0 > $O/seq.json 2> $O/seq.err || { tail -5 $O/seq.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/seq.json')); print('line', d['value'], d['ms_per_step']); print(json.dumps(d['w_hc_seq'], indent=1))"
