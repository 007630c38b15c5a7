#!/bin/bash
# One GPU-box pass over the round's gates: the GPU parity suite, smoke(), the 1-GPU bench (driver contract) and the
# --gpus 2 launch rehearsed with gloo on the box's one GPU.  Every GPU step has its own time limit; the chain stops at
# the first failure.   TAG=<name> names the outputs under gpurun_out/.
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-chk}
mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest_gpu.log 2>&1 \
  || { tail -40 $OUT/${TAG}_pytest_gpu.log; exit 1; }
tail -2 $OUT/${TAG}_pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { tail -20 $OUT/${TAG}_smoke.log; exit 1; }
tail -1 $OUT/${TAG}_smoke.log
timeout -k 10 400 python bench.py ${BENCH_ARGS} > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { tail -20 $OUT/${TAG}_bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${TAG}_bench.json')); print('C2 %.4gM poses/s kernel %.4f ms; C3 %.4gM gicp %.2f ms' % (d['value']/1e6, d['roofline']['kernel_ms'], d['c3']['value']/1e6, d['c3']['gicp']['gicp_ms_per_step']))"
PCORE_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --no-cpu --c3-steps 1 > $OUT/${TAG}_bench_gpus2.json 2> $OUT/${TAG}_bench_gpus2.err \
  || { tail -20 $OUT/${TAG}_bench_gpus2.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$OUT/${TAG}_bench_gpus2.json') if l.startswith('{')][-1]); print('gpus2 n_gpus', d['n_gpus'], 'value %.4gM' % (d['value']/1e6), d['config'])"
