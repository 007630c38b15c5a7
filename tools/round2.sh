#!/bin/bash
# New GPU tests (full-size properties), the bench with its CPU legs, a 2-rank gloo rehearsal of the
# multi-rank bench on one GPU, and the C1 GPU config.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-r01c}
mkdir -p $OUT; export TMPDIR=/tmp
echo "== fullsize tests"
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_full_$TAG.log 2>&1 || { tail -40 $OUT/pytest_full_$TAG.log; exit 1; }
tail -8 $OUT/pytest_full_$TAG.log
echo "== bench"
timeout -k 10 600 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
echo "== 2-rank gloo rehearsal"
PCORE_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > $OUT/bench2_$TAG.json 2> $OUT/bench2_$TAG.err || { tail -20 $OUT/bench2_$TAG.err; exit 1; }
cat $OUT/bench2_$TAG.json
echo "== C1 GPU"
timeout -k 10 300 python tools/bench_configs.py --configs C1 > $OUT/c1_$TAG.jsonl 2> $OUT/c1_$TAG.err || { tail -20 $OUT/c1_$TAG.err; exit 1; }
cat $OUT/c1_$TAG.jsonl
