# process-to-process spread of the gradient kernel: 8 separate bench processes each for grad_variant 0 and 5
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/s3d; mkdir -p $O; cd $R
for i in 1 2 3 4 5 6 7 8; do
  timeout -k 10 200 python bench.py --no-cpu --steps 4 --warmup 2 > $O/b0_$i.json 2> $O/b0_$i.err && \
  timeout -k 10 200 python bench.py --no-cpu --steps 4 --warmup 2 --tune grad_variant=5 > $O/b5_$i.json 2> $O/b5_$i.err || break
done
echo rc=$?
for f in $O/b*_*.json; do python -c "
import json; d=json.load(open('$f')); a=d['alloc']; print('$f'.split('/')[-1], d['ms_per_step'], d['kernels']['grad']['avg_ms'], d['kernels']['log_softmax']['avg_ms'], d['roofline']['box_copy_gbps'], hex(a['acts']), hex(a['grads']))"; done
