set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "icp" -x -q --timeout 300 --timeout-method thread > gpurun_out/r03f_icp.log 2>&1 && \
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03f_phase.txt 2>&1 && \
LIBS="build_ab/dppred.so build_ab/lanepar.so build_ab/dppred.so build_ab/lanepar.so" TESTK="icp" bash tools/c3_ab.sh > gpurun_out/r03f_c3ab.txt 2>&1
