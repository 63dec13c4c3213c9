#!/bin/bash
# Stall breakdown of the inflate kernel: one rocprofv3 --pmc pass per counter
# group over the bench workload at --repeats ${REPEATS:-40} (the hardware cannot multiplex; at most
# 8 SQ + 2 GRBM counters per pass).  Outputs gpurun_out/stall_<g>/ ; tools/stall_summary.py turns
# them into profiles/<tag>_inflate_stalls.json.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=${REPEATS:-40}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/rocprof_counters.txt 2>&1 || true
run() {
  g=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" -d gpurun_out/stall_$g -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api --repeats $R > gpurun_out/stall_$g.log 2>&1 || exit $?
}
run A SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
run B SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU
run C SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT
run D SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES SQ_LDS_IDX_ACTIVE SQ_IFETCH
run E SQ_INST_LEVEL_LDS SQ_ACCUM_PREV_HIRES SQ_INSTS_LDS
