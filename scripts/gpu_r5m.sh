#!/bin/bash
# Round 5: NoisySimulator through the in-tile path — tests, then 26q W-HC noisy line tile vs pulled.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${1:-r5m}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu -x tests/test_noisy_gpu.py > $O/pytest_noisy.log 2>&1 || { tail -30 $O/pytest_noisy.log; exit 1; }
tail -1 $O/pytest_noisy.log
for t in 1 0; do
  QSIM_NOISY_TILE=$t timeout -k 10 300 python -u bench.py --workload noisy --cpu-budget 0 --steps 3 > $O/noisy$t.json 2> $O/noisy$t.err || { tail -5 $O/noisy$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/noisy$t.json'));print('noisy tile=$t', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),4), k['launches']) for k in d['kernels']], [(k['name'], round(k['ms']/max(1,k['launches']),4)) for k in d['kernels_overlapped']])"
done
