set -o pipefail
mkdir -p gpurun_out/r04pp
timeout -k 10 400 python3 -u tools/ab_multi.py --rounds 3 --steps 3 cur=abtmp/cur/libppgpu.so wgrp=abtmp/wgrp/libppgpu.so noprio=abtmp/noprio/libppgpu.so wgrpnp=abtmp/wgrpnp/libppgpu.so > gpurun_out/r04pp/ab.json 2> gpurun_out/r04pp/ab.log || { rc=$?; tail -20 gpurun_out/r04pp/ab.log; exit $rc; }
grep '^\[ab\]' gpurun_out/r04pp/ab.log | tail -12
