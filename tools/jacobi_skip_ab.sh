set -o pipefail
KERNEL=covariance_cloud TAG=r06l2 LIBS="build_ab/jskip1.so build_ab/jskip2.so build_ab/covskip1b.so" bash tools/gicp_lib_ab.sh
