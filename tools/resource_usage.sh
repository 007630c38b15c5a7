#!/bin/bash
# Registers, spills, scratch and LDS of the GICP / fused kernels as the compiler reports them (no GPU needed):
#   tools/resource_usage.sh [extra hipcc flags, e.g. -DPCORE_GICP_LDS_ROUNDS=1]
cd "$(dirname "$0")/.."
FLAGS=$(python -c "from perception_amd import build; print(' '.join(f for f in build.flags() if f not in ('-shared','-fPIC')))")
for SRC in pcore_gicp.hip pcore_kernels.hip; do
  /opt/rocm/bin/hipcc $FLAGS "$@" --offload-device-only -S perception_amd/csrc/$SRC -o /dev/null \
    -Rpass-analysis=kernel-resource-usage 2>&1 | python -c "
import re, sys
cur = None
for l in sys.stdin:
    m = re.search(r'remark: Function Name: (\S+)', l)
    if m:
        cur = m.group(1); continue
    m = re.search(r'remark:\s+(VGPRs|VGPRs Spill|SGPRs Spill|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)', l)
    if m and cur and ('gicp_kernel' in cur or 'fused_cost' in cur or 'covariance_kernel' in cur):
        print(f'{cur[:60]:60s} {m.group(1):28s} {m.group(2)}')
"
done
