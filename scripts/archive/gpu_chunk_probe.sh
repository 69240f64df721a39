#!/bin/bash
set -o pipefail
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/chunk; mkdir -p $O
for U in 0 22; do QSIM_CHUNK_QUBITS=$U timeout -k 10 120 python scripts/dbg/chunk_check.py 26 || exit 1; done
for nt in 1 0; do for U in 0 20 22 23 24; do
  QSIM_JIT_NT=$nt QSIM_CHUNK_QUBITS=$U timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-budget 0 --no-1q28 > $O/hc_${nt}_$U.json || exit 1
  python3 -c "
import json; d=json.load(open('$O/hc_${nt}_$U.json'))
print('NT=$nt U=$U', d['value'], d['ms_per_step'], [(k['name'], round(k['ms']/max(1,k['launches']),3), k['launches']) for k in d['kernels']])"
done; done
