#!/bin/bash
# Build an A/B variant of libpcore.so into build_ab/NAME.so with extra compiler flags (defines), on the CPU:
#   tools/build_variant.sh NAME [-DFOO=1 ...]
# Load it with PCORE_LIB=$PWD/build_ab/NAME.so (tools/lib_ab.sh, tools/fused_phase_prof.py, ...).
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
mkdir -p build_ab
FLAGS=$(python -c "from perception_amd import build; print(' '.join(build.flags()))")
SRCS=$(python -c "from perception_amd import build; import os; print(' '.join(os.path.join(build.CSRC, f) for f in build.SOURCES))")
/opt/rocm/bin/hipcc $FLAGS "$@" $SRCS -o build_ab/$NAME.so
echo build_ab/$NAME.so
