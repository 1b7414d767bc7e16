#!/bin/bash
# SQ / LDS counter passes over the step's kernels (through gpurun): where each MFMA or gather kernel's
# wave cycles go (parked on s_waitcnt / barrier, issue-stalled, issuing), how busy the matrix pipe is,
# LDS bank conflicts.  Eager steps (rocprofv3 sees every dispatch), one counter set per pass, each
# pass under its own time limit; stops at the first pass that does not end cleanly.
#   TAG=r4x bash scripts/pmc_sq.sh [list]
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$(pwd)
TAG=${TAG:-r4}
KRE=${KRE:-'chain_fwd_v4_ln|chain_bwd_v3|conv_proj_fwd|conv_proj_bwd_gate|feat_fwd|tiled_flat|attn_fwd_center_sf|attn_bwd_center|sbf_radial_wgrad'}
if [ "${1:-}" = "list" ]; then
  timeout -s KILL 120 rocprofv3 -L > gpurun_out/counters_$TAG.txt 2>&1
  echo "list rc=$?"
fi
pass() {  # pass <name> <counters...>
  local name=$1; shift
  echo "=== pmc $name: $*"
  timeout -s KILL 240 rocprofv3 --pmc "$@" --kernel-include-regex "$KRE" -d "gpurun_out/pmc_${name}_$TAG" -o run \
    --output-format csv -- python "$ROOT/bench.py" --step-only --eager --steps 3 --warmup 1 ${BARGS:-} \
    > "gpurun_out/pmc_${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  tail -n 3 "gpurun_out/pmc_${name}_$TAG.log"
  [ $rc -eq 0 ] || exit $rc
}
pass sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass sqb SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD \
  SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE
python scripts/pmc_sq_summary.py gpurun_out/pmc_sqa_$TAG gpurun_out/pmc_sqb_$TAG > gpurun_out/pmc_sq_$TAG.txt 2>&1
cat gpurun_out/pmc_sq_$TAG.txt
