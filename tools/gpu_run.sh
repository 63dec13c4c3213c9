#!/bin/bash
# One gpurun call's worth of GPU work, as named steps (replaces r01-r04's one-off run scripts):
#
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash tools/gpu_run.sh <tag> <step> [<step> ...]
#
# Every step runs under its own time limit, writes under gpurun_out/<tag>/, and the first failing
# step ends the call (a GPU fault, abort or time limit is never followed by more GPU work).
# Steps:
# A step may carry arguments after ':' -- for gputest a -k selection with ',' for " or ", for the
# bench steps extra bench.py arguments with '_' for a space (e.g. stamps:--share_8).
#   gputest[:<k1,k2,...>]       pytest -m gpu (all, or the tests matching any k)   -> gputest.txt
#   smoke                       __graft_entry__.smoke()                            -> smoke.txt
#   bench                       the default bench line (python bench.py)           -> bench_default.json
#   profile                     rocprofv3 kernel stats + FETCH/WRITE passes, summarised into
#                               profiles/<tag>_bench*.{json,csv} and profiles/traffic.json
#   stalls                      the stall PMC passes -> profiles/<tag>_inflate_stalls.json + inflate_stalls.json
#   create_index                GPU CreateIndex of the 50 GB member                -> create_index.json
#   paired                      configs[4]'s 2 x 25 GB pair on one GPU             -> paired.json
#   w8                          bench.py --gpus 8 on ONE GPU (gloo + host transport) at the real
#                               50 GB member ($W8_ARGS appended)                    -> w8.json
#   shares                      N = 1 and rank 0's share of N = $SHARES (default "2 4 8"); variants
#                               $VARIANTS = "tag:args" items ('_' = space)         -> shares/*.json
#   ab                          tools/ab_multi.py over $AB_BUILDS ("tag=lib ...")   -> ab.json
#   stamps[:args]               the PPG_STAMPS diagnostic build (abtmp/stamps) on the bench workload
#                               (e.g. stamps:--share_8)                            -> stamps*.log
#   chunkapi                    the per-chunk Decompress leg only ($CHUNK_ARGS)    -> chunkapi.json
#   latency[:args]              tools/chunk_latency.py with every launch's phases  -> chunk_latency.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
[ -n "$tag" ] || { echo "usage: gpu_run.sh <tag> <step>..." >&2; exit 2; }
O=gpurun_out/$tag
mkdir -p "$O"
NOLEGS="--no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api"
line() {   # the bench line's headline numbers
  python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; print(sys.argv[1], round(d['value']/1e6,2), d.get('unit'), round(d['ms_per_step'],2), 'ms', d.get('kernel_ms_per_step'), (d.get('roofline') or {}).get('frac'))" "$1"
}
run_step() {
  local step=$1 arg=${1#*:} xa
  [ "$arg" = "$step" ] && arg=""
  xa=${arg//_/ }
  case ${step%%:*} in
  gputest)
    if [ -n "$arg" ]; then sel=(-k "${arg//,/ or }"); else sel=(); fi
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread "${sel[@]}" > $O/gputest.txt 2>&1
    rc=$?; tail -2 $O/gputest.txt
    [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gputest.txt | head -20; return $rc; } ;;
  smoke)
    timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -5 $O/smoke.txt; return 1; }
    tail -1 $O/smoke.txt ;;
  bench)
    timeout -k 10 500 python3 -u bench.py $xa > $O/bench_default.json 2> $O/bench_default.log || return $?
    line $O/bench_default.json ;;
  profile)
    bash tools/profile_round.sh || return $?
    python3 tools/traffic_summary.py $tag > $O/traffic_summary.txt 2>&1 || return $?
    cp profiles/${tag}_* profiles/traffic.json $O/ 2>/dev/null
    rm -rf gpurun_out/prof_stats gpurun_out/prof_FETCH_SIZE gpurun_out/prof_WRITE_SIZE ;;
  stalls)
    bash tools/pmc_stalls.sh || return $?
    python3 tools/stall_summary.py $tag > $O/stall_summary.txt 2>&1 || return $?
    cp profiles/${tag}_inflate_stalls.json profiles/inflate_stalls.json $O/ 2>/dev/null
    rm -rf gpurun_out/stall_? ;;
  create_index)
    timeout -k 10 300 python3 -u bench.py --create-index --steps 2 --warmup 1 $NOLEGS > $O/create_index.json 2> $O/create_index.log || return $?
    tail -c 400 $O/create_index.json ;;
  paired)
    timeout -k 10 400 python3 -u bench.py --paired --steps 3 --warmup 1 $PAIRED_ARGS > $O/paired.json 2> $O/paired.log || return $?
    line $O/paired.json ;;
  w8)
    # (r06: with the N > 1 end-to-end leg; --no-ingest in W8_ARGS skips it)
    PPG_BENCH_ONE_DEVICE=1 PPG_DIST_BACKEND=gloo timeout -k 10 900 python3 -u bench.py --gpus 8 --steps 2 --warmup 1 \
      --no-cpu-baseline --no-enumerate --no-chunk-api $W8_ARGS $xa > $O/w8.json 2> $O/w8.log || { tail -20 $O/w8.log; return 1; }
    line $O/w8.json ;;
  shares)
    mkdir -p $O/shares
    if [ -z "$SKIP_N1" ]; then
      timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 $NOLEGS > $O/shares/n1.json 2> $O/shares/n1.log || return $?
      line $O/shares/n1.json
    fi
    for n in ${SHARES-2 4 8}; do
      timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 $NOLEGS --share $n > $O/shares/share$n.json 2> $O/shares/share$n.log || return $?
      line $O/shares/share$n.json
    done
    for spec in $VARIANTS; do
      a=${spec#*:}
      timeout -k 10 300 python3 -u bench.py --steps ${STEPS:-5} --warmup 2 $NOLEGS ${a//_/ } > $O/shares/v_${spec%%:*}.json 2> $O/shares/v_${spec%%:*}.log || return $?
      line $O/shares/v_${spec%%:*}.json
    done ;;
  e2eshares)   # rank 0's share of an N-way split, resident AND end to end from a file (r06)
    mkdir -p $O/shares
    for n in ${SHARES-2 4 8}; do
      timeout -k 10 400 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --share $n $xa > $O/shares/e2e$n.json 2> $O/shares/e2e$n.log || return $?
      line $O/shares/e2e$n.json
      python3 -c "import json,sys; d=[json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]; i=d.get('ingest',{}); print({k: i.get(k) for k in ('records_per_s','compressed_GBps','seconds_max_over_ranks','piece_GiB','waves_per_chunk','error')})" $O/shares/e2e$n.json
    done ;;
  ab)
    timeout -k 10 900 python3 -u tools/ab_multi.py $AB_ARGS $AB_BUILDS > $O/ab.json 2> $O/ab.log || { tail -5 $O/ab.log; return 1; }
    tail -c 1500 $O/ab.json ;;
  stamps)
    [ -f abtmp/stamps/ppg_inflate.lint ] || { echo "stamps: build abtmp/stamps first (tools/ab_build.sh stamps -DPPG_STAMPS)"; return 3; }
    local st=stamps${arg:+_${arg//[^a-z0-9]/}}
    PPG_LIB_PATH=abtmp/stamps/libppgpu.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 $NOLEGS $xa \
      > $O/$st.json 2> $O/$st.log || return $?
    grep PPG_STAMPS $O/$st.log | tail -4 ;;
  chunkapi)
    timeout -k 10 400 python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-enumerate $xa \
      > $O/chunkapi.json 2> $O/chunkapi.log || return $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); c=d.get('decompress_chunk', {}); print(json.dumps(c)[:1500])" $O/chunkapi.json ;;
  latency)
    PPG_CHUNK_VERBOSE=1 timeout -k 10 300 python3 -u tools/chunk_latency.py $xa > $O/chunk_latency.txt 2>&1 || { tail -5 $O/chunk_latency.txt; return 1; }
    grep -v PPG_CHUNK $O/chunk_latency.txt | tail -14 ;;
  *)
    echo "gpu_run.sh: unknown step $step" >&2; return 2 ;;
  esac
}
for st in "$@"; do
  echo "== $tag: $st ($(date +%T))"
  run_step "$st" || { rc=$?; echo "== $tag: step $st failed (exit $rc): stopping"; exit $rc; }
done
du -sh gpurun_out
exit 0
