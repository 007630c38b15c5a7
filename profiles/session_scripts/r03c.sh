set -o pipefail
mkdir -p gpurun_out
PCORE_LIB=$PWD/build_ab/gprof.so timeout -k 10 200 python -u tools/gicp_phase_prof.py --c3 > gpurun_out/r03c_phase.txt 2>&1
