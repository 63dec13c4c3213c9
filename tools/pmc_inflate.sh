#!/bin/bash
# SQ counter passes over the inflate kernel (bench workload at --repeats ${REPEATS:-40}), one
# rocprofv3 --pmc pass per counter group (the hardware cannot multiplex): gpurun_out/pmc_<g>/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
R=${REPEATS:-40}
run() {
  g=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d gpurun_out/pmc_$g -o pmc --output-format csv -- \
    python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --repeats $R > gpurun_out/pmc_$g.log 2>&1 || exit $?
}
run A SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES
run B SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC
run C SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE GRBM_COUNT
