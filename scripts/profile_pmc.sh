#!/bin/bash
# rocprofv3 PMC counters for the headline force kernel (kernel-trace + pmc only; no sys/runtime
# trace in the same run). Writes gpurun_out/pmc_*/ ; summarise with scripts/pmc_summary.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
run() {  # $1 = tag, rest = counters
  tag=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc_$tag -o pmc --output-format csv \
    -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmc_$tag.log 2>&1
}
run valu SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE || exit $?
run cycles SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY || exit $?
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 || exit $?
exit 0
