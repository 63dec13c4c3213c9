set -o pipefail
mkdir -p gpurun_out
# 1. same-box A/B of the SALU-cut variants (one process, one resident member)
timeout -k 10 600 python3 -u tools/ab_multi.py --rounds 3 --steps 3 base=abtmp/base/libppgpu.so lim=abtmp/lim/libppgpu.so limsgb=abtmp/limsgb/libppgpu.so hot=abtmp/hot/libppgpu.so ispec=abtmp/ispec/libppgpu.so hotis=abtmp/hotis/libppgpu.so widx=abtmp/widx/libppgpu.so carry=abtmp/carry/libppgpu.so hotl=abtmp/hotl/libppgpu.so hotlwc=abtmp/hotlwc/libppgpu.so all=abtmp/all/libppgpu.so hota=abtmp/hota/libppgpu.so hotlwa=abtmp/hotlwa/libppgpu.so hotlwt8=abtmp/hotlwt8/libppgpu.so hotlwta8=abtmp/hotlwta8/libppgpu.so rb11=abtmp/base/libppgpu.so,PPG_RING_BITS=11 > gpurun_out/r04_abm.json 2> gpurun_out/r04_abm.log || { rc=$?; tail -20 gpurun_out/r04_abm.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04_abm.log | tail -25
# 2. the chunk service (found side points) first, then the whole GPU suite
timeout -k 10 240 python -u -m pytest tests/test_gpu_chunk_threads.py -v -s --timeout 200 --timeout-method thread > gpurun_out/r04_gputest_chunk.txt 2>&1 || { rc=$?; tail -30 gpurun_out/r04_gputest_chunk.txt; exit $rc; }
grep -E "found\]|passed|failed" gpurun_out/r04_gputest_chunk.txt | tail -5
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r04_gputest_full.txt 2>&1
rc=$?; tail -3 gpurun_out/r04_gputest_full.txt
case $rc in 0|1) ;; *) echo "suite rc=$rc: stopping"; exit $rc;; esac
timeout -k 10 300 python -u bench.py --paired --steps 3 --warmup 1 > gpurun_out/r04_paired.json 2> gpurun_out/r04_paired.log || exit $?
grep '^{' gpurun_out/r04_paired.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('paired', d['value']/1e6, 'Mpairs/s', d['ms_per_step'], d['config']['pair_check'])"
