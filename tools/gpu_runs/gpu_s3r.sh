# per-buffer write rates by pattern (grid-stride, whole 4 KiB rows per wave in order / scattered, scattered
# 2 MiB pages): is the slow-write buffer class slow for every pattern?
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3r; mkdir -p $O; cd $R
for i in 1 2 3; do
  timeout -k 10 300 ./tools/membench --buffers 4 48 16 > $O/mb_$i.json 2> $O/mb_$i.err || break
done
echo rc=$?
for i in 1 2 3; do python -c "
import json; d=json.load(open('$O/mb_$i.json'))
for b in d['buffers']: print('proc $i rnt %.0f wnt %.0f w %.0f rows %.0f rows_sc %.0f pages_sc %.0f' % (b['read_nt'], b['write_nt'], b['write'], b['write_rows'], b['write_rows_scattered'], b['write_pages_scattered']))"; done
