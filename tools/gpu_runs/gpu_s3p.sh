# per-buffer HBM streaming rates: 4 buffers of 48 GiB, whole-buffer read/write/copy and per-4-GiB write rates,
# three processes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3p; mkdir -p $O; cd $R
for i in 1 2 3; do
  timeout -k 10 300 ./tools/membench --buffers 4 48 4 > $O/mb_$i.json 2> $O/mb_$i.err || break
done
echo rc=$?
for i in 1 2 3; do python -c "
import json; d=json.load(open('$O/mb_$i.json'))
for b in d['buffers']: print('proc $i', b['ptr'], 'rnt %.0f r %.0f wnt %.0f w %.0f cp %.0f' % (b['read_nt'], b['read'], b['write_nt'], b['write'], b['copy_in_nt']), 'sub', b['sub_write_nt'])"; done
