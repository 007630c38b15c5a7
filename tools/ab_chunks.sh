set -o pipefail
export TMPDIR=/tmp
PCORE_STREAM_CHUNKS=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tier or evaluate_costs or edge or sampled or fixture or random_pose or icp_sweep" > gpurun_out/pt_ch4.log 2>&1 || { tail -30 gpurun_out/pt_ch4.log; exit 1; }
tail -1 gpurun_out/pt_ch4.log
for r in 1 2; do for C in 1 4 8; do
  PCORE_STREAM_CHUNKS=$C timeout -k 10 300 python tools/bench_configs.py --configs C2,C3 --steps 10 | cut -c1-200 | sed "s/^/ch=$C /" || exit 1
done; done
