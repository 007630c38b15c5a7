export TMPDIR=/tmp
timeout -k 10 500 python -m pytest tests -q -x -m gpu -k "icp or recognizer" > gpurun_out/icp_pytest.log 2>&1; r=$?; tail -5 gpurun_out/icp_pytest.log; [ $r = 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/icpw -o run -- python tools/prof_fused.py --iters 2 --icp > gpurun_out/icpw.log 2>&1 || exit 1
python -c "
import csv
for r in csv.reader(open('gpurun_out/icpw/run_kernel_stats.csv')): print(r[0][:40], r[1:4])"
TAG=sqg ARGS="--icp --iters 1" bash tools/sq_counters.sh || exit 1
for i in 0 1 2; do python tools/pmc_summary.py gicp_kernel gpurun_out/sqg_$i/run_counter_collection.csv; done > gpurun_out/sqg_summary.txt
