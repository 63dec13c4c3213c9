#!/bin/bash
# one SQ instruction-mix pass over the inflate kernel (bench workload at --repeats ${REPEATS:-40})
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES \
  -d gpurun_out/pmc_q${TAG} -o pmc --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --repeats ${REPEATS:-40} \
  > gpurun_out/pmc_q${TAG}.log 2>&1
