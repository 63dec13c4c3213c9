set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04u
# the default bench line on the round's final tree (the driver's command)
timeout -k 10 500 python3 -u bench.py > gpurun_out/r04u/bench_default.json 2> gpurun_out/r04u/bench_default.log || { rc=$?; tail -20 gpurun_out/r04u/bench_default.log; exit $rc; }
tail -c 900 gpurun_out/r04u/bench_default.json
