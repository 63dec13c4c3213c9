set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04p
# the pipelined build's parity (the whole GPU suite + smoke), then pipe vs bperm-before-finish
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04p/gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/r04p/gputest.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/r04p/gputest.txt | head -20; exit $rc; }
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04p/smoke.txt 2>&1 || { tail -5 gpurun_out/r04p/smoke.txt; exit 1; }
tail -1 gpurun_out/r04p/smoke.txt
timeout -k 10 500 python3 -u tools/ab_multi.py --rounds 3 --steps 3 pipe=abtmp/pipe/libppgpu.so pbp=abtmp/pbp/libppgpu.so pbp3=abtmp/pbp3/libppgpu.so p2=abtmp/p2/libppgpu.so p2b=abtmp/p2b/libppgpu.so p3=abtmp/p3/libppgpu.so > gpurun_out/r04l_ab.json 2> gpurun_out/r04l_ab.log || { rc=$?; tail -20 gpurun_out/r04l_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04l_ab.log | tail -18
