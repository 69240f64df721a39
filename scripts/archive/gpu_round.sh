#!/bin/bash
# One gpurun call: GPU tests, benches (20/28/30q + 28q W-1Q), rocprof kernel stats at 30q, PMC traffic at 30q + 28q.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R && ONEQ=1 PROF=1 TAG=${TAG:-run} bash scripts/gpu_validate.sh && \
  cd $R && QUBITS=30 TAG=${TAG:-run}_30 bash scripts/gpu_pmc.sh && \
  cd $R && QUBITS=28 TAG=${TAG:-run}_28 bash scripts/gpu_pmc.sh && \
  cd $R && QUBITS=28 WORKLOAD=1q TAG=${TAG:-run}_28_1q bash scripts/gpu_pmc.sh
