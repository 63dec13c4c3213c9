set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04r
# the first 32 KiB of every chunk / piece through the pipelined loop too (PPG_EARLYPIPE): the whole
# GPU suite on that build, then same-box timings against the shipped build
PPG_LIB_PATH=abtmp/ep/libppgpu.so timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04r/ep_gputest.txt 2>&1
rc=$?; tail -2 gpurun_out/r04r/ep_gputest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04r/ep_gputest.txt | head -20; exit $rc; }
timeout -k 10 300 python3 -u tools/ab_multi.py --rounds 3 --steps 3 cur=abtmp/cur2/libppgpu.so ep=abtmp/ep/libppgpu.so > gpurun_out/r04r/ab.json 2> gpurun_out/r04r/ab.log || { rc=$?; tail -20 gpurun_out/r04r/ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04r/ab.log | tail -6
for t in cur2 ep; do
  for n in 8 4; do
    PPG_LIB_PATH=abtmp/$t/libppgpu.so timeout -k 10 300 python3 -u bench.py --share $n --steps 5 --warmup 2 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/r04r/share${n}_$t.json 2> gpurun_out/r04r/share${n}_$t.log || exit $?
    python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04r/share${n}_$t.json') if l.startswith('{')][-1]; print('share$n $t', round(d['ms_per_step'],2), d['kernel_ms_per_step'])"
  done
  PPG_LIB_PATH=abtmp/$t/libppgpu.so timeout -k 10 300 python3 -u bench.py --create-index --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-enumerate --no-chunk-api > gpurun_out/r04r/ci_$t.json 2> gpurun_out/r04r/ci_$t.log || exit $?
  python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04r/ci_$t.json') if l.startswith('{')][-1]; c=d['create_index']; print('ci $t', round(c['seconds'],3), c['phases_ms']['pass1_ms'], c['phases_ms']['pass2_ms'])"
done
