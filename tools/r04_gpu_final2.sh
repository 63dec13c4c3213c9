set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04y
# r04 final build (pipelined far load, token lookup before the finish, stream DMA after it):
# parity first, then the unrolled-walk A/B, the round profiles (summarised on the box), the
# default line and the N = 8 strong share
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04y/gputest.txt 2>&1
rc=$?; tail -2 gpurun_out/r04y/gputest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04y/gputest.txt | head -20; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04y/smoke.txt 2>&1 || { tail -5 gpurun_out/r04y/smoke.txt; exit 1; }
tail -1 gpurun_out/r04y/smoke.txt
timeout -k 10 300 python3 -u tools/ab_multi.py --rounds 3 --steps 3 cur=abtmp/cur/libppgpu.so fin=abtmp/fin/libppgpu.so > gpurun_out/r04y/ab.json 2> gpurun_out/r04y/ab.log || { rc=$?; tail -20 gpurun_out/r04y/ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04y/ab.log | tail -6
bash tools/profile_round.sh || exit $?
bash tools/pmc_stalls.sh || exit $?
python3 tools/traffic_summary.py r04y > gpurun_out/r04y/traffic_summary.txt 2>&1 || exit $?
python3 tools/stall_summary.py r04y > gpurun_out/r04y/stall_summary.txt 2>&1 || exit $?
cp profiles/r04y_* profiles/traffic.json profiles/inflate_stalls.json gpurun_out/r04y/
rm -rf gpurun_out/prof_stats gpurun_out/prof_FETCH_SIZE gpurun_out/prof_WRITE_SIZE gpurun_out/stall_?
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04y/bench_default.json 2> gpurun_out/r04y/bench_default.log || exit $?
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04y/bench_default.json') if l.startswith('{')][-1]; print(d['value']/1e6, d['ms_per_step'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['roofline']['issue'] and d['roofline']['issue']['salu_per_cu_cycle'])"
SKIP_W8=1 STEPS=5 SHARES="2 4 8" bash tools/r04_shares.sh || exit $?
mkdir -p gpurun_out/r04y/shares && mv gpurun_out/r04_n1.* gpurun_out/r04_share*.* gpurun_out/r04y/shares/
du -sh gpurun_out
