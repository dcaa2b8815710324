# gradient-kernel time vs the relative placement of grads and acts, in one process (kbench grads_offset_kb),
# repeated in two processes; then two bench processes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3f; mkdir -p $O; cd $R
V='[{"grads_offset_kb":0},{"grads_offset_kb":4},{"grads_offset_kb":64},{"grads_offset_kb":1024},{"grads_offset_kb":2048},{"grads_offset_kb":2052},{"grads_offset_kb":4096},{"grads_offset_kb":16384},{"grads_offset_kb":32768},{"grads_offset_kb":262144},{"grads_offset_kb":524288},{"grads_offset_kb":1048576}]'
for i in 1 2 3; do
  timeout -k 10 400 python tools/kbench.py --ws-first --rounds 3 --variants "$V" > $O/kb_$i.json 2> $O/kb_$i.err || break
done
echo rc=$?
for i in 1 2 3; do python -c "
import json; d=json.load(open('$O/kb_$i.json')); print('proc $i', d['alloc'])
print(' '.join('%s:%.2f/%.2f' % (v['knobs']['grads_offset_kb'], v['median_ms']['grad'], v['median_ms']['log_softmax']) for v in d['variants']))"; done
