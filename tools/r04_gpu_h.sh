set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 4 --steps 3 r4f=abtmp/r4f/libppgpu.so wgrp=abtmp/wgrp/libppgpu.so wgrpp2=abtmp/wgrpp2/libppgpu.so prio2=abtmp/prio2/libppgpu.so > gpurun_out/r04h_ab.json 2> gpurun_out/r04h_ab.log || { rc=$?; tail -20 gpurun_out/r04h_ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04h_ab.log | tail -16
