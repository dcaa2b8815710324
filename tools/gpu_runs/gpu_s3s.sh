# buffer write-rate classes with contiguous vs scattered (2 MiB pieces) physical backing; also the torch
# caching allocator with expandable segments (buffers mapped in 20 MiB segments)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3s; mkdir -p $O; cd $R
for i in 1 2 3; do
  timeout -k 10 300 ./tools/membench --buffers 3 40 40 > $O/mb_plain_$i.json 2> $O/mb_plain_$i.err && \
  timeout -k 10 300 ./tools/membench --buffers 3 40 40 100 > $O/mb_frag_$i.json 2> $O/mb_frag_$i.err || break
done
for i in 1 2 3; do
  PYTORCH_HIP_ALLOC_CONF=expandable_segments:True timeout -k 10 300 python tools/kbench.py --ws-first --rounds 3 --buffers 2 --variants '[{},{"grads_buf":1,"acts_buf":1}]' > $O/kb_exp_$i.json 2> $O/kb_exp_$i.err || break
done
echo rc=$?
for f in $O/mb_*.json; do python -c "
import json; d=json.load(open('$f'))
print('$f'.split('/')[-1], ' | '.join('rnt %.0f wnt %.0f' % (b['read_nt'], b['write_nt']) for b in d['buffers']))"; done
for i in 1 2 3; do python -c "
import json; d=json.load(open('$O/kb_exp_$i.json'))
print('expandable $i', [{k:round(x,3) for k,x in v['median_ms'].items()} for v in d['variants']])"; done
