set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "icp or color" -x -v --timeout 200 --timeout-method thread > gpurun_out/r03a_icp.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -k "c3" -x -v --timeout 250 --timeout-method thread > gpurun_out/r03a_c3.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_configs.py --configs C3 --steps 3 --warmup 1 > gpurun_out/r03a_c3.jsonl 2>&1 && \
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
