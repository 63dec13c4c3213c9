set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04f
# r04 final build: round profiles (rocprof stats, FETCH/WRITE, stall passes) summarised ON the box
# (the raw per-dispatch CSVs exceed gpurun_out's 64 MiB), then the default bench line, which picks
# up the build-pinned traffic and stall files, and the strong-scaling shares
bash tools/profile_round.sh || exit $?
bash tools/pmc_stalls.sh || exit $?
python3 tools/traffic_summary.py r04 > gpurun_out/r04f/traffic_summary.txt 2>&1 || exit $?
python3 tools/stall_summary.py r04 > gpurun_out/r04f/stall_summary.txt 2>&1 || exit $?
cp profiles/r04_* profiles/traffic.json profiles/inflate_stalls.json gpurun_out/r04f/
cp gpurun_out/prof_stats.json gpurun_out/prof_stats.log gpurun_out/stall_A.log gpurun_out/r04f/ 2>/dev/null
rm -rf gpurun_out/prof_stats gpurun_out/prof_FETCH_SIZE gpurun_out/prof_WRITE_SIZE gpurun_out/stall_? 
timeout -k 10 400 python3 -u bench.py > gpurun_out/r04f/bench_default.json 2> gpurun_out/r04f/bench_default.log || exit $?
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/r04f/bench_default.json') if l.startswith('{')][-1]; print(d['value']/1e6, d['ms_per_step'], d['kernel_ms_per_step'], d['roofline'])"
SKIP_W8=1 STEPS=5 bash tools/r04_shares.sh || exit $?
mkdir -p gpurun_out/r04f/shares && mv gpurun_out/r04_n1.* gpurun_out/r04_share*.* gpurun_out/r04f/shares/
du -sh gpurun_out
