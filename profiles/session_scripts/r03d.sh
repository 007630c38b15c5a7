set -o pipefail
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03c_phase.txt 2>&1 && \
LIBS="build_ab/disc.so build_ab/mask.so" MASKS="0 1 2 4 8" bash tools/lds_conflicts.sh > gpurun_out/r03d_ldsc.txt 2>&1 && \
LIBS="build_ab/disc.so build_ab/mask.so build_ab/disc.so build_ab/mask.so" CONFIGS=C2,C5 bash tools/lib_ab.sh > gpurun_out/r03d_ab.txt 2>&1
