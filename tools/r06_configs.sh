#!/bin/bash
# Round 6 wider measurements: every BASELINE config through tools/bench_configs.py (C1..C5 and the scan meshes; C3's
# ADD-S AUC), the drop-in recognizer end to end, and the GPU's GICP (cycle exit on) against the independent numpy
# chain run to 150 iterations on 1,000 candidates.  Each step under its own limit; TAG names the outputs.
set -o pipefail
OUT=gpurun_out/${TAG:-cfg}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u tools/bench_configs.py --configs C1,C2,C3,C4,C5,C2scan_blob,C2scan_shell,C3scan > $OUT/configs.jsonl 2> $OUT/configs.err \
  || { tail -20 $OUT/configs.err; exit 1; }
python -c "
import json
for l in open('$OUT/configs.jsonl'):
    d = json.loads(l); print(d['config'], '%.4g poses/s' % d['poses_per_s'], 'auc', d.get('adds_auc'), 'gicp mean', d.get('gicp_iters_mean'))"
timeout -k 10 600 python -u tools/recognizer_e2e.py > $OUT/recognizer_e2e.txt 2>&1 || { tail -20 $OUT/recognizer_e2e.txt; exit 1; }
tail -6 $OUT/recognizer_e2e.txt
timeout -k 10 900 python -u tools/gpu_vs_independent.py --poses-per-object 200 --out $OUT/gpu_vs_independent_1000.json > $OUT/gpu_vs_independent.log 2>&1 \
  || { tail -20 $OUT/gpu_vs_independent.log; exit 1; }
cat $OUT/gpu_vs_independent_1000.json
