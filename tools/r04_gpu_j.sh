set -o pipefail
mkdir -p gpurun_out
# the pipelined far load: records checked against the member's count inside ab_multi, then a
# golden-parity run of the variant through the test suite's shard path
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 3 --steps 3 r4f=abtmp/r4f/libppgpu.so pipe=abtmp/pipe/libppgpu.so > gpurun_out/r04j_ab.json 2> gpurun_out/r04j_ab.log || { rc=$?; tail -20 gpurun_out/r04j_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04j_ab.log | tail -8
