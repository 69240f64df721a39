timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_batched_refnoise_gpu.py > gpurun_out/rn.log 2>&1; tail -5 gpurun_out/rn.log
