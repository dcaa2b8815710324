# gradient-kernel speed vs which physical buffers hold acts / grads: two of each in one process, all four
# pairings, four processes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3j; mkdir -p $O; cd $R
V='[{},{"grads_buf":1},{"acts_buf":1},{"acts_buf":1,"grads_buf":1}]'
for i in 1 2 3 4; do
  timeout -k 10 300 python tools/kbench.py --ws-first --rounds 3 --buffers 2 --variants "$V" > $O/kb_$i.json 2> $O/kb_$i.err || break
done
echo rc=$?
for i in 1 2 3 4; do python -c "
import json; d=json.load(open('$O/kb_$i.json')); a=d['alloc']
print('proc $i', [hex(x) for x in a['acts_bufs']], [hex(x) for x in a['grads_bufs']])
for v in d['variants']: print('   ', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
