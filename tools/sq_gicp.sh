#!/bin/bash
# SQ counter passes over the GICP kernel on C3 (counters only, no trace domains; the last pass is the f64 /
# transcendental instruction mix for the cycle-weighted VALU figure); the iteration count of the
# profiled calls goes to $OUT/${TAG}_iters.json for tools/sq_gicp_json.py.
set -o pipefail
OUT=${OUT:-gpurun_out}; TAG=${TAG:-sqg}
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 GRBM_GUI_ACTIVE"; do
  timeout -k 10 300 rocprofv3 --pmc $SET --kernel-trace --output-format csv -d $OUT/${TAG}_$i -o run -- python tools/prof_fused.py --c3 --icp --iters 1 --iters-json $OUT/${TAG}_iters.json > $OUT/${TAG}_$i.log 2>&1 || { tail -20 $OUT/${TAG}_$i.log; exit 1; }
  i=$((i+1))
done
echo ok
