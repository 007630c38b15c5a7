set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS="build_ab/lanepar.so build_ab/upiv.so build_ab/lds0.so build_ab/lanepar.so build_ab/upiv.so build_ab/lds0.so" TESTK="icp" bash tools/c3_ab.sh > gpurun_out/r03g_c3ab.txt 2>&1 && \
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03g_phase.txt 2>&1
