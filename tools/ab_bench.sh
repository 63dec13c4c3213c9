#!/bin/bash
# A/B timing of libppgpu.so variants on the GPU box: tools/ab_bench.sh <tag> <lib.so> [<tag> <lib.so> ...]
# Each variant runs the default bench workload (50 GB member, resident) without the CPU baseline;
# output: gpurun_out/ab_<tag>.json (+ .log).  Stops at the first failing run.
set -o pipefail
mkdir -p gpurun_out
while [ $# -ge 2 ]; do
  tag=$1; lib=$2; shift 2
  # a variant built outside the default make must have passed the inline-asm wait-state lint
  # (tools/hazard_lint.py writes ppg_inflate.lint next to the objects only when it is clean)
  if [ "$(dirname "$lib")" != "parallelparsing_amd" ] && [ ! -f "$(dirname "$lib")/ppg_inflate.lint" ]; then
    echo "ab_bench: $lib has no clean ppg_inflate.lint beside it; refusing to run it" >&2; exit 3
  fi
  PPG_LIB_PATH=$lib timeout -k 10 300 python -u bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-cpu-baseline --no-ingest ${AB_ARGS} \
    > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.log || exit $?
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$tag.json')); print('$tag', round(d['value']/1e6,1), 'Mrec/s', {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()})"
done
