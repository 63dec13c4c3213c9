#!/bin/bash
# A/B timing of libppgpu.so variants on the GPU box: tools/ab_bench.sh <tag> <lib.so> [<tag> <lib.so> ...]
# Each variant runs the default bench workload (50 GB member, resident) without the CPU baseline;
# output: gpurun_out/ab_<tag>.json (+ .log).  Stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  tag=$1; lib=$2; shift 2
  PPG_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-cpu-baseline --no-ingest ${AB_ARGS} \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.log || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', round(d['value']/1e6,1), 'Mrec/s', {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"
done
