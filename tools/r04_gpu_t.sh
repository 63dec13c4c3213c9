set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04t
# A/B of the block finder prefilter (BFINAL = 0 or not) on the per-chunk Decompress leg, alternating on one box
for r in 1 2; do for b in old new; do
  PPG_LIB_PATH=abtmp/$b/libppgpu.so timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ingest --no-enumerate > gpurun_out/r04t/${b}_$r.json 2> gpurun_out/r04t/${b}_$r.log || exit $?
  python3 -c "
import json; d=[json.loads(l) for l in open('gpurun_out/r04t/${b}_$r.json') if l.startswith('{')][-1]
print('$b $r', {k: (round(v['records_per_s']/1e6,2), round(v['ms_per_call'],2)) for k,v in d['decompress_chunk'].items() if isinstance(v,dict) and 'records_per_s' in v})"
done; done
