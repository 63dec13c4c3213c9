#!/bin/bash
# r02 measurement pass (run on the GPU box through gpurun):
#   1. FETCH_SIZE calibration (tools/fetch_calib: known bytes, 4 access patterns)
#   2. SQ instruction mix of the inflate kernel (bench workload at --repeats 40)
#   3. A/B timing at the full 50 GB step: the default kernel vs the kernel without the fused census
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib -o calib --output-format csv -- ./tools/fetch_calib \
  > gpurun_out/calib.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM \
  SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_mix -o pmc --output-format csv -- python3 bench.py --steps 1 \
  --warmup 0 --no-cpu-baseline --no-ingest --repeats 40 > gpurun_out/pmc_mix.json 2> gpurun_out/pmc_mix.log || exit $?
AB_STEPS=3 bash tools/ab_bench.sh base parallelparsing_amd/libppgpu.so || exit $?
PPG_PROBE_NO_CENSUS=1 AB_STEPS=3 bash tools/ab_bench.sh nocensus parallelparsing_amd/libppgpu.so || exit $?
