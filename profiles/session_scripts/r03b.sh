set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03b_phase.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03b_c3prof -o run -- python tools/prof_fused.py --c3 --icp --iters 3 > gpurun_out/r03b_c3prof.log 2>&1 && \
OUT=gpurun_out TAG=sqg bash tools/sq_gicp.sh > gpurun_out/r03b_sqg.log 2>&1
