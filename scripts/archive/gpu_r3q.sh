#!/bin/bash
# Round 3: default bench line (with roofline_batch16) + PMC of the reference-noise W-BATCH.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r3q
mkdir -p $O
timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_batched_gpu.py tests/test_api_gpu.py tests/test_tile13_gpu.py tests/test_sampling_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --cpu-budget 0 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));b=d['roofline_batch16'];print(d['value'], d['roofline']['frac'], {k:(b[k]['value'],b[k]['ms_per_step'],b[k]['roofline']['kernel'],b[k]['roofline']['frac']) for k in ('reference','physical')})"
cd /tmp
for i in 1 2; do
  C=FETCH_SIZE; [ $i = 2 ] && C=WRITE_SIZE
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/pmc/p$i -o run --output-format csv -- python3 $R/bench.py --workload batch --batch-noise reference --steps 1 --warmup 0 --cpu-budget 0 > $O/pmc_p$i.log 2>&1 || { tail -5 $O/pmc_p$i.log; exit 1; }
done
python3 $R/scripts/pmc_summary.py $O/pmc $O/pmc_batch_ref_16q.json
