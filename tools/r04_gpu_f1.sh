set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
# r04 final build: the whole GPU suite + smoke, a last same-box A/B, the round profiles
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04f_gputest.txt 2>&1
rc=$?; tail -3 gpurun_out/r04f_gputest.txt
case $rc in 0|1) ;; *) echo "suite rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04f_smoke.txt 2>&1 || { tail -5 gpurun_out/r04f_smoke.txt; exit 1; }
tail -2 gpurun_out/r04f_smoke.txt
timeout -k 10 300 python3 -u tools/ab_multi.py --rounds 3 --steps 3 r4f=abtmp/r4f/libppgpu.so prio2=abtmp/prio2/libppgpu.so base=abtmp/base/libppgpu.so > gpurun_out/r04f_ab.json 2> gpurun_out/r04f_ab.log || { rc=$?; tail -20 gpurun_out/r04f_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04f_ab.log | tail -9
bash tools/profile_round.sh || exit $?
bash tools/pmc_stalls.sh || exit $?
echo done
