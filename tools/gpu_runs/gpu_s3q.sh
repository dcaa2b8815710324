# staged gradient: nontemporal vs plain stores / loads, two buffer pairs, two processes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3q; mkdir -p $O; cd $R
V='[{},{"nt_store":0},{"nt_load":0},{"grads_buf":1,"acts_buf":1},{"grads_buf":1,"acts_buf":1,"nt_store":0},{"grads_buf":1,"acts_buf":1,"nt_load":0}]'
for i in 1 2; do
  timeout -k 10 300 python tools/kbench.py --ws-first --rounds 3 --buffers 2 --variants "$V" > $O/kb_$i.json 2> $O/kb_$i.err || break
done
echo rc=$?
for i in 1 2; do python -c "
import json; d=json.load(open('$O/kb_$i.json'))
print('proc $i')
for v in d['variants']: print('   ', v['knobs'], {k:round(x,3) for k,x in v['median_ms'].items()})"; done
