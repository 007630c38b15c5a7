set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03e_phase.txt 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "icp or color" -x -q --timeout 200 --timeout-method thread > gpurun_out/r03e_icp.log 2>&1 && \
LIBS="build_ab/disc.so build_ab/mask.so" MASKS="0 1 2 4 8" bash tools/lds_conflicts.sh > gpurun_out/r03e_ldsc.txt 2>&1 && \
LIBS="build_ab/mask.so build_ab/dppred.so build_ab/lmpf.so build_ab/mask.so build_ab/dppred.so build_ab/lmpf.so" TESTK="icp" bash tools/c3_ab.sh > gpurun_out/r03e_c3ab.txt 2>&1 && \
LIBS="build_ab/disc.so build_ab/mask.so build_ab/disc.so build_ab/mask.so" CONFIGS=C2,C5 bash tools/lib_ab.sh > gpurun_out/r03e_ab.txt 2>&1 && \
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -k "full or share or gloo" -x -v --timeout 600 --timeout-method thread > gpurun_out/r03e_fullsize.log 2>&1
