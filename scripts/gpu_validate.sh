set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; echo pytest_rc=$?; tail -3 gpurun_out/pytest_gpu.log
for n in 28 30; do
  timeout -k 10 300 python bench.py --qubits $n --steps 5 --warmup 1 --cpu-budget 10 > gpurun_out/bench$n.json 2> gpurun_out/bench$n.err || { echo bench$n failed; exit 1; }
done
timeout -k 10 300 python bench.py --qubits 28 --workload 1q --steps 2 --warmup 1 --cpu-budget 0 > gpurun_out/bench28_1q.json 2> gpurun_out/bench28_1q.err || exit 1
timeout -k 10 300 python bench.py --qubits 28 --mode per-gate --steps 2 --warmup 1 --cpu-budget 0 > gpurun_out/bench28_pergate.json 2> gpurun_out/bench28_pergate.err || exit 1
echo done
