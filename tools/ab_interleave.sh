#!/bin/bash
# Interleaved A/B of libppgpu.so variants on one GPU box: tools/ab_interleave.sh <rounds> <tag>=<lib>[,VAR=val...] ...
# Each round runs every variant once (default bench workload, resident 50 GB member, no CPU
# baseline / ingest), so box drift hits every variant alike.  Output gpurun_out/abi_<tag>_<round>.json
# and one summary line per run; variants built outside the default make need a clean
# ppg_inflate.lint beside them (tools/ab_build.sh).
set -o pipefail
mkdir -p gpurun_out
rounds=$1; shift
for ((i = 1; i <= rounds; i++)); do
  for spec in "$@"; do
    tag=${spec%%=*}; rest=${spec#*=}; lib=${rest%%,*}; envs=""
    [ "$rest" != "$lib" ] && envs=${rest#*,}
    if [ "$(dirname "$lib")" != "parallelparsing_amd" ] && [ ! -f "$(dirname "$lib")/ppg_inflate.lint" ]; then
      echo "ab_interleave: $lib has no clean ppg_inflate.lint beside it" >&2; exit 3
    fi
    env ${envs//,/ } PPG_LIB_PATH=$lib timeout -k 10 300 python3 -u bench.py --steps ${AB_STEPS:-3} --warmup 1 \
      --no-cpu-baseline --no-ingest --no-chunk-api ${AB_ARGS} > gpurun_out/abi_${tag}_$i.json 2> gpurun_out/abi_${tag}_$i.log || exit $?
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/abi_${tag}_$i.json') if l.startswith('{')][-1]); print('$tag', $i, round(d['value']/1e6,1), 'Mrec/s', {k: round(v,1) for k,v in d['kernel_ms_per_step'].items()}, d['build']['build_id'])"
  done
done
